"""The ABI's largest accepted P (2^30 columns: every per-row byte offset, and
a row's buffer-descriptor range, at the 32-bit limit) through each layout and
column mapping: sampled columns, including the last ones, against the oracle
bit for bit.  About 20 GB of HBM."""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref

pytestmark = pytest.mark.gpu

P = 1 << 30
K = 2


@pytest.fixture(scope="module")
def data():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fedsim_amd import ops

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2024)
    X = torch.empty((K, P), dtype=torch.float32, device=dev).uniform_(-1, 1, generator=g)
    w = [3, 7]
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    rng = np.random.default_rng(5)
    cols = np.unique(np.concatenate([rng.integers(0, P, 4096), np.arange(P - 4100, P),
                                     np.arange(0, 64)]))
    idx = torch.from_numpy(cols).to(dev)
    Xs = X[:, idx].cpu().numpy()
    want = ref.reduce(np.ascontiguousarray(Xs), w, W=sum(w))
    yield dict(dev=dev, X=X, w=w, w32=w32, idx=idx, want=want)
    del X
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mapping", ["auto", "wide", "narrow1", "narrow2", "narrow4"])
@pytest.mark.parametrize("layout", ["strided", "rows"])
def test_max_P(layout, mapping, data):
    from fedsim_amd import ops

    d = data
    out = torch.empty(P, dtype=torch.float32, device=d["dev"])
    fl = ops.tuning_flags(mapping=mapping)
    if layout == "strided":
        ops.reduce_slab(d["X"], d["w32"], out, W=sum(d["w"]), flags=fl)
    else:
        ops.reduce_rows([d["X"][0], d["X"][1]], d["w32"], out, W=sum(d["w"]), flags=fl)
    got = out[d["idx"]].cpu().numpy()
    np.testing.assert_array_equal(bits(got), bits(d["want"]))
    del out


def test_max_P_blocked_fused_step(data):
    """The column-blocked slab and the fused FedAvg step at P = 2^30."""
    from fedsim_amd import ops

    d = data
    Xb = ops.to_blocked(d["X"], 4096)
    cloud = torch.zeros(P, dtype=torch.float32, device=d["dev"])
    step = ops.ServerStep("fedavg", cloud, lr=1.0)
    ops.reduce_blocked_step(Xb, d["w32"], step, W=sum(d["w"]))
    del Xb
    got = cloud[d["idx"]].cpu().numpy()
    zero = np.zeros_like(d["want"])
    np.testing.assert_array_equal(bits(got), bits(ref.fedavg_sgd(d["want"], zero, 1.0)))


@pytest.mark.parametrize("kcap", [(1 << 18) - 1, 1 << 18])
def test_blocked_region_at_the_descriptor_limit(kcap):
    """A column block's region (Kcap * C * 4 bytes) just under 4 GiB takes the
    buffer-descriptor kernels, at 4 GiB the flat ones; rows at the very end of
    the region, both column blocks (one ragged), against the oracle."""
    from fedsim_amd import ops
    from oracle import vectors as V

    dev = torch.device("cuda:0")
    C, Pc, B = 4096, 4096 + 5, 3
    X = V.client_rows("realistic", B, Pc, 17)
    w = V.client_weights("fedavg", B, 17)
    Xb = torch.empty(ops.blocked_shape(kcap, Pc, C), dtype=torch.float32, device=dev)
    r0 = kcap - B
    for j in range(B):
        ops.pack_row(torch.from_numpy(X[j].copy()).to(dev), Xb, r0 + j)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    out = torch.empty(Pc, dtype=torch.float32, device=dev)
    want = ref.reduce(X, w, W=sum(w))
    for mapping in ("auto", "wide", "narrow4"):
        ops.reduce_blocked(Xb, w32, out, B=B, W=sum(w), r0=r0,
                           flags=ops.tuning_flags(mapping=mapping))
        np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(want))
    del Xb
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kcap", [(1 << 18) - 1, 1 << 18])
def test_blocked_full_region_high_row_offsets(kcap):
    """Every row of a region just under / at 4 GiB (row offsets up to ~4 GiB
    in the 32-bit soffset), values in {0, 1} and weights 1 so that every
    partial sum is an integer below 2^24 and the result is known exactly."""
    from fedsim_amd import ops

    dev = torch.device("cuda:0")
    C, Pc = 4096, 4096 + 5
    nb = 2
    Xb = torch.empty((nb, kcap, C), dtype=torch.float32, device=dev)
    k = torch.arange(kcap, dtype=torch.int32, device=dev).view(-1, 1)
    for b in range(nb):
        p = (b * C + torch.arange(C, dtype=torch.int32, device=dev)).view(1, -1)
        Xb[b] = ((7 * k + p) % 3 == 0).float()
    del k
    w32 = torch.ones(kcap, dtype=torch.float32, device=dev)
    cols = np.arange(Pc)
    # k = -p (mod 3) for k in [0, kcap)
    res = (-cols) % 3
    count = (kcap - 1 - res) // 3 + 1
    want = (count.astype(np.float32) / np.float32(kcap)).astype(np.float32)
    out = torch.empty(Pc, dtype=torch.float32, device=dev)
    for mapping in ("auto", "wide", "narrow4"):
        ops.reduce_blocked(Xb, w32, out, W=kcap, flags=ops.tuning_flags(mapping=mapping))
        np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(want))
    del Xb
    torch.cuda.empty_cache()


def test_max_P_tile_rows(data):
    """The largest P that takes fedagg_reduce_rows_f32's wide-tile path
    (2^30 - 4: P = 2^30 itself keeps the flat-load narrow kernel): the
    sampled columns against the oracle, with the divide."""
    from fedsim_amd import ops

    P2 = P - 4
    rows = [data["X"][k, :P2] for k in range(K)]
    out = torch.empty(P2, dtype=torch.float32, device=data["dev"])
    ops.reduce_rows(rows, data["w32"], out, W=sum(data["w"]))
    keep = (data["idx"] < P2).cpu().numpy()
    got = out[data["idx"][data["idx"] < P2]].cpu().numpy()
    np.testing.assert_array_equal(bits(got), bits(data["want"][keep]))


@pytest.mark.parametrize("dtype,P_big", [("bfloat16", (1 << 31) + 7), ("float64", (1 << 29) + 3)])
def test_generic_kernel_rows_over_4_GiB(dtype, P_big):
    """fedagg_reduce_rows_ref with rows of more than 4 GiB (64-bit element
    offsets, the wide tile and the scalar tail): sampled columns, the last
    ones included, bitwise the reference's CPU arithmetic on them."""
    from fedsim_amd import ops
    from oracle.reference_loop import ReferenceSerialAggregator

    dt = getattr(torch, dtype)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(77)
    rows = [torch.empty(P_big, dtype=dt, device=dev).uniform_(-1, 1, generator=g)
            for _ in range(2)]
    w = [3, 0.37]
    out = torch.empty(P_big, dtype=dt, device=dev)
    ops.reduce_rows_ref(rows, w, out)
    rng = np.random.default_rng(8)
    cols = np.unique(np.concatenate([rng.integers(0, P_big, 4096), np.arange(P_big - 70, P_big)]))
    idx = torch.from_numpy(cols).to(dev)
    ref_agg = ReferenceSerialAggregator()
    for r, wk in zip(rows, w):
        ref_agg.add("p", r[idx].cpu(), wk)
    ib = torch.int64 if dt == torch.float64 else torch.int16
    assert torch.equal(out[idx].cpu().view(ib), ref_agg.get_sum("p").view(ib))
    del rows, out
    torch.cuda.empty_cache()
