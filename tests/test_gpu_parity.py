"""GPU parity: the HIP path (through the C-ABI) vs the reference's golden
outputs and the pinned oracle.  Bar: bit-exact (exact mode)."""
import numpy as np
import pytest
import torch

from conftest import bits, golden_cases
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu

CASES = golden_cases()
PARAM_CASES = [c for c in CASES if all(c["ok"]) and c["has_params"] and "opts" not in c]
# "default" lets the library pick the column mapping (narrow at these sizes);
# the others force the wide f32x4-slot kernels or a narrow (one / two columns
# per lane) one with a given unroll
VARIANTS = {
    "default": dict(),
    "u4v2nt": dict(unroll=4, vpt=2, nt=True, mapping="wide"),
    "u8v1": dict(unroll=8, vpt=1, mapping="wide"),
    "u16v2": dict(unroll=16, vpt=2, mapping="wide"),
    "u4v1nt": dict(unroll=4, vpt=1, nt=True, mapping="wide"),
    "n1u8nt": dict(unroll=8, nt=True, mapping="narrow1"),
    "n1u32": dict(unroll=32, mapping="narrow1"),
    "n2u16nt": dict(unroll=16, nt=True, mapping="narrow2"),
    "n2u8": dict(unroll=8, mapping="narrow2"),
    "n4u8nt": dict(unroll=8, nt=True, mapping="narrow4"),
    "n4u32": dict(unroll=32, mapping="narrow4"),
}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fedsim_amd import _native

    _native.load()
    return torch.device("cuda:0")


def _inputs(case):
    X = V.client_rows(case["dist"], case["K"], case["P"], case["seed"])
    assert V.sha256(X) == case["input_sha256"]
    return X


def _expect(case, arrays, name, got):
    assert V.sha256(got) == case["outputs_sha256"][name], f"{case['id']}:{name}"
    if case["stored"]:
        np.testing.assert_array_equal(bits(got), bits(arrays[f"{case['id']}/{name}"]))


@pytest.mark.parametrize("variant", list(VARIANTS))
@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_reduce_slab_bitwise(case, variant, dev, golden):
    from fedsim_amd import ops

    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, _ = ref.accepted(case["weights"])
    Xd = torch.from_numpy(np.ascontiguousarray(X[idx])).to(dev)
    w32 = torch.tensor([ops.fl32(w) for w in ws], dtype=torch.float32, device=dev)
    out = torch.empty(case["P"], dtype=torch.float32, device=dev)
    fl = ops.tuning_flags(**VARIANTS[variant])
    ops.reduce_slab(Xd, w32, out, flags=fl)
    _expect(case, arrays, "sum", out.cpu().numpy())
    ops.reduce_slab(Xd, w32, out, W=W, flags=fl)
    _expect(case, arrays, "avg", out.cpu().numpy())


@pytest.mark.parametrize("mapping", ["auto", "wide", "narrow2", "narrow4"])
@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_reduce_rows_and_batches_bitwise(case, mapping, dev, golden):
    """Row-table kernel, and the reduction split into batches chained through
    the accumulator, both equal the single-pass reference result."""
    from fedsim_amd import ops

    fl = ops.tuning_flags(mapping=mapping)

    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, _ = ref.accepted(case["weights"])
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in idx]
    w32 = torch.tensor([ops.fl32(w) for w in ws], dtype=torch.float32, device=dev)
    out = torch.empty(case["P"], dtype=torch.float32, device=dev)
    ops.reduce_rows(rows, w32, out, W=W, flags=fl)
    _expect(case, arrays, "avg", out.cpu().numpy())
    # batches of 1, 2, 3, ... rows, finalize fused into the last batch
    acc = torch.empty_like(out)
    k0, b = 0, 1
    first = True
    while k0 < len(rows):
        k1 = min(len(rows), k0 + b)
        last = k1 == len(rows)
        ops.reduce_rows(rows[k0:k1], w32[k0:k1].contiguous(), acc,
                        acc_in=None if first else acc, W=W if last else None, flags=fl)
        first, k0, b = False, k1, b + 1
    _expect(case, arrays, "avg", acc.cpu().numpy())


@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_epilogues_bitwise(case, dev, golden):
    from fedsim_amd import ops

    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, _ = ref.accepted(case["weights"])
    avg = torch.from_numpy(ref.reduce(X[idx], ws, W=W)).to(dev)
    cloud0 = V.cloud_vector(case["P"], case["seed"] + 1)
    for lr in case["lrs"]:
        cloud = torch.from_numpy(cloud0.copy()).to(dev)
        if case["algo"] == "adabest":
            prev = torch.from_numpy(V.cloud_vector(case["P"], case["seed"] + 2)).to(dev)
            ops.adabest_sgd(avg, cloud, prev, case["beta"], lr)
            _expect(case, arrays, f"avg_params_lr{lr}", prev.cpu().numpy())
        elif case["algo"] == "feddyn":
            h = torch.from_numpy(V.cloud_vector(case["P"], case["seed"] + 3)).to(dev)
            ap = torch.empty_like(h)
            ops.feddyn_sgd(avg, cloud, h, W / case["num_clients"], lr, avg_prev=ap)
            _expect(case, arrays, f"h_lr{lr}", h.cpu().numpy())
            _expect(case, arrays, f"avg_params_lr{lr}", ap.cpu().numpy())
        else:
            ops.fedavg_sgd(avg, cloud, lr)
        _expect(case, arrays, f"cloud_lr{lr}", cloud.cpu().numpy())


def test_scalar_path_unaligned_rows(dev):
    """Rows at a 4-byte (not 16-byte) offset take the generic kernel; same bits."""
    from fedsim_amd import ops

    K, P = 9, 1029
    X = V.client_rows("normal", K, P + 1, 77)
    w = V.client_weights("fedavg", K, 77)
    big = torch.from_numpy(X).to(dev)
    rows = [big[k, 1:] for k in range(K)]  # 4-byte misaligned views
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    ops.reduce_rows(rows, w32, out, W=sum(w))
    exp = ref.reduce(np.ascontiguousarray(X[:, 1:]), w, W=sum(w))
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(exp))
    ops.reduce_slab(big[:, 1:], w32, out, W=sum(w))
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(exp))


def test_empty_inputs(dev):
    from fedsim_amd import ops

    w32 = torch.ones(1, dtype=torch.float32, device=dev)
    # B = 0: writes +0.0 (and 0/W when finalizing)
    out = torch.full((37,), 5.0, device=dev)
    ops.reduce_slab(torch.empty((0, 37), device=dev), w32, out)
    assert torch.equal(out.cpu(), torch.zeros(37))
    # P = 0: no launch, no error
    ops.reduce_slab(torch.empty((3, 0), device=dev), w32.repeat(3), torch.empty(0, device=dev))


@pytest.mark.parametrize("C", [1024, 2048, 4096])
@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_reduce_blocked_bitwise(case, C, dev, golden):
    """Column-blocked slab layout (packed with the 2-D DMA), whole slab and as
    a ring drained in two row ranges, equals the reference bitwise."""
    from fedsim_amd import ops

    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, _ = ref.accepted(case["weights"])
    B, P = len(idx), case["P"]
    Xb = torch.full(ops.blocked_shape(B + 3, P, C), float("nan"), device=dev)
    host = torch.from_numpy(np.ascontiguousarray(X[idx])).pin_memory()
    for j in range(B):  # rows 2..B+1 of a B+3-row slab; odd rows from the host
        src = host[j] if j % 2 else host[j].to(dev)
        ops.pack_row(src, Xb, j + 2)
    w32 = torch.tensor([ops.fl32(w) for w in ws], dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    for variant in ("default", "u4v2nt", "u8v1", "n1u8nt", "n2u16nt", "n2u8", "n4u8nt"):
        fl = ops.tuning_flags(**{k: v for k, v in VARIANTS[variant].items() if k != "vpt"})
        ops.reduce_blocked(Xb, w32, out, B=B, W=W, flags=fl, r0=2)
        _expect(case, arrays, "avg", out.cpu().numpy())
    h = B // 2
    ops.reduce_blocked(Xb, w32[:h].contiguous(), out, B=h, r0=2)
    ops.reduce_blocked(Xb, w32[h:].contiguous(), out, B=B - h, acc_in=out, W=W, r0=2 + h)
    _expect(case, arrays, "avg", out.cpu().numpy())


def test_pack_row_layout(dev):
    from fedsim_amd import ops

    for P in (1, 5, 4095, 4096, 4097, 9000):
        K, C = 3, 4096
        X = torch.randn(K, P)
        Xb = torch.zeros(ops.blocked_shape(K, P, C), device=dev)
        srcs = [X[k].contiguous().pin_memory() for k in range(K)]  # alive until synced
        for k in range(K):
            ops.pack_row(srcs[k], Xb, k)
        torch.cuda.synchronize()
        ref_b = ops.to_blocked(X.to(dev), C)
        assert torch.equal(Xb, ref_b)
        # HBM -> HBM pack (copy kernel) and unaligned device source (DMA path)
        Xb2 = torch.zeros_like(Xb)
        Xd = X.to(dev)
        for k in range(K):
            ops.pack_row(Xd[k].contiguous(), Xb2, k)
        assert torch.equal(Xb2, ref_b)
        if P > 1:
            Xu = torch.zeros(K, P + 1, device=dev)
            Xu[:, 1:] = Xd
            Xb3 = torch.zeros(ops.blocked_shape(K, P, C), device=dev)
            for k in range(K):
                ops.pack_row(Xu[k, 1:], Xb3, k)  # 4-byte aligned source
            assert torch.equal(Xb3, ref_b)


@pytest.mark.parametrize("mapping", ["auto", "wide", "narrow1", "narrow2", "narrow4"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9, 255, 256, 257, 1022, 1025])
def test_mappings_small_and_ragged_P(P, mapping, dev):
    """Every column mapping at sizes around its per-lane width and workgroup
    span (the two- and four-column kernels fall back when P does not divide),
    with acc_in chaining, against the oracle."""
    from fedsim_amd import ops

    K = 7
    X = V.client_rows("normal", K, P, 31 + P)
    w = V.client_weights("fedavg", K, 31 + P)
    Xd = torch.from_numpy(X).to(dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    fl = ops.tuning_flags(mapping=mapping)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    ops.reduce_slab(Xd[:3], w32[:3], out, flags=fl)
    ops.reduce_slab(Xd[3:], w32[3:].contiguous(), out, acc_in=out, W=sum(w), flags=fl)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.reduce(X, w, W=sum(w))))


@pytest.mark.parametrize("mapping", ["narrow2", "narrow4"])
def test_mappings_misaligned_operands(mapping, dev):
    """Rows, accumulator and output at 4- and 8-byte offsets: the wider narrow
    kernels step down to what the alignment allows; same bits."""
    from fedsim_amd import ops

    K, P = 6, 4100
    X = V.client_rows("realistic", K, P + 2, 5)
    w = V.client_weights("fedavg", K, 5)
    W = sum(w)
    big = torch.from_numpy(X).to(dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    fl = ops.tuning_flags(mapping=mapping)
    for off in (1, 2):
        rows = big[:, off:off + P]
        want = ref.reduce(np.ascontiguousarray(X[:, off:off + P]), w, W=W)
        buf = torch.empty(P + 4, dtype=torch.float32, device=dev)
        out = buf[off:off + P]
        ops.reduce_slab(rows[:2], w32[:2], out, flags=fl)
        ops.reduce_slab(rows[2:], w32[2:].contiguous(), out, acc_in=out, W=W, flags=fl)
        np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(want))
        tab_rows = [rows[k] for k in range(K)]
        out2 = torch.empty(P, dtype=torch.float32, device=dev)
        ops.reduce_rows(tab_rows, w32, out2, W=W, flags=fl)
        np.testing.assert_array_equal(bits(out2.cpu().numpy()), bits(want))
