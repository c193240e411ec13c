"""Property-based GPU parity (hypothesis): random client counts, sizes, value
ranges, weight kinds, column-block widths, slab capacities and ring splits,
every layout and the fused pop + step, against the C oracle.

Bar: bit-exact for finite results.  Where an input overflow makes inf - inf,
both sides produce a NaN, but its sign/payload is not pinned (x86's default
NaN is negative, CDNA's is positive). Those positions are compared as "NaN
on both sides", and every other position bit for bit.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import bits
from oracle import ref
from test_oracle_properties import rounds

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]

SETTINGS = settings(max_examples=250, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow,
                                           HealthCheck.function_scoped_fixture])


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fedsim_amd import _native

    _native.load()
    return torch.device("cuda:0")


def same(got, exp):
    got = np.asarray(got, dtype=np.float32)
    nan_g, nan_e = np.isnan(got), np.isnan(exp)
    np.testing.assert_array_equal(nan_g, nan_e)
    np.testing.assert_array_equal(bits(got[~nan_g]), bits(exp[~nan_e]))


def _accepted(X, w):
    keep = [k for k in range(len(w)) if w[k] > 0]
    return X[keep], [w[k] for k in keep]


@SETTINGS
@given(rounds(max_k=40, max_p=9000), st.sampled_from([1024, 2048, 4096]),
       st.integers(0, 5), st.data())
def test_blocked_ring_random(dev, r, C, pad, data):
    from fedsim_amd import ops

    X, w = r
    Xa, wa = _accepted(X, w)
    B, P = len(wa), X.shape[1]
    if B == 0:
        return
    W = sum(wa)
    Xb = ops.to_blocked(torch.from_numpy(Xa).to(dev), C, kcap=B + pad)
    w32 = torch.tensor([ops.fl32(v) for v in wa], dtype=torch.float32, device=dev)
    out = torch.empty(P, device=dev)
    cut = data.draw(st.integers(0, B))
    if cut:
        ops.reduce_blocked(Xb, w32[:cut].contiguous(), out, B=cut)
    ops.reduce_blocked(Xb, w32[cut:].contiguous(), out, B=B - cut,
                       acc_in=out if cut else None, W=W, r0=cut)
    exp = ref.reduce(Xa, wa, W=W)
    same(out.cpu().numpy(), exp)


@SETTINGS
@given(rounds(max_k=20, max_p=5000), st.sampled_from(["fedavg", "adabest", "feddyn"]),
       st.sampled_from([0.0, 0.9]), st.floats(0.05, 1.5))
def test_fused_step_random(dev, r, algo, m, lr):
    from fedsim_amd import ops

    X, w = r
    Xa, wa = _accepted(X, w)
    B, P = len(wa), X.shape[1]
    if B == 0:
        return
    W = sum(wa)
    avg = ref.reduce(Xa, wa, W=W)
    rng = np.random.default_rng(P + B)
    cloud0 = rng.normal(0, 0.05, P).astype(np.float32)
    aux0 = rng.normal(0, 0.05, P).astype(np.float32) if algo != "fedavg" else None
    s = ref.ServerState(algo, cloud0, dict(lr=lr, momentum=m), aux=aux0, coef=0.6)
    s.step(avg)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    aux = torch.from_numpy(aux0.copy()).to(dev) if aux0 is not None else None
    buf = torch.empty(P, device=dev) if m else None
    grad = torch.empty(P, device=dev)
    step = ops.ServerStep(algo, cloud, lr=lr, momentum=m, coef=0.6, aux=aux, momentum_buf=buf,
                          momentum_init=bool(m), grad_out=grad)
    C = ops.choose_block_cols(P)
    Xb = ops.to_blocked(torch.from_numpy(Xa).to(dev), C)
    w32 = torch.tensor([ops.fl32(v) for v in wa], dtype=torch.float32, device=dev)
    ops.reduce_blocked_step(Xb, w32, step, W=W)
    same(cloud.cpu().numpy(), s.cloud)
    same(grad.cpu().numpy(), s.grad)
    if aux is not None:
        same(aux.cpu().numpy(), s.aux)
    if m:
        same(buf.cpu().numpy(), s.buf)


@SETTINGS
@given(rounds(max_k=24, max_p=3000), st.integers(1, 9))
def test_aggregator_random_stream(dev, r, max_rows):
    """add() x K through a small ring, host sources into one key and HBM
    sources into another (one key holds one device, as the reference's
    running sum does), then pop()."""
    from fedsim_amd.utils import SerialAggregator

    X, w = r
    agg = SerialAggregator(max_rows=max_rows)
    for k in range(X.shape[0]):
        src = torch.from_numpy(X[k].copy())
        agg.add("h", src, w[k])
        agg.add("d", src.to(dev), w[k])
    if X.shape[0] == 0:
        assert "h" not in agg and "d" not in agg
        return
    W = sum(w)  # add() does not skip zero weights; W == 0 -> pop returns the raw sum
    want = ref.reduce(X, w, W=W if W else None)
    got_h, got_d = agg.pop("h"), agg.pop("d")
    assert got_h.device.type == "cpu" and got_d.device == dev
    same(got_h.numpy(), want)
    same(got_d.cpu().numpy(), want)


@pytest.mark.parametrize("C", [1024, 4096])
def test_nonfinite_inputs(dev, C):
    """+-inf and NaN client values (a diverged client the caller did not flag)
    propagate as in the reference: inf stays inf with its sign, inf - inf and
    NaN inputs give NaN at exactly the same positions."""
    from fedsim_amd import ops

    K, P = 6, 5000
    rng = np.random.default_rng(17)
    X = rng.standard_normal((K, P)).astype(np.float32)
    X[0, :100] = np.inf
    X[1, 50:150] = -np.inf          # inf - inf in columns 50..99
    X[2, 200:220] = np.nan
    X[3, 300:310] = np.float32(3e38)  # overflows to inf once weighted
    w = [3, 1, 2, 7, 5, 4]
    W = sum(w)
    Xb = ops.to_blocked(torch.from_numpy(X).to(dev), C)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    out = torch.empty(P, device=dev)
    ops.reduce_blocked(Xb, w32, out, W=W)
    exp = ref.reduce(X, w, W=W)
    assert np.isnan(exp[50:100]).all() and np.isposinf(exp[:50]).all()
    same(out.cpu().numpy(), exp)


@SETTINGS
@given(rounds(max_k=40, max_p=6000),
       st.sampled_from(["wide", "narrow1", "narrow2", "narrow4"]),
       st.sampled_from([0, 8, 16, 32]), st.sampled_from(["strided", "rows", "blocked"]),
       st.integers(0, 3))
def test_mapping_random(dev, r, mapping, unroll, layout, split):
    """Every column mapping x unroll x layout on random shapes and values,
    split into two chained calls at a random row, against the oracle."""
    from fedsim_amd import ops

    X, w = _accepted(*r)
    K, P = X.shape
    if K == 0:
        return
    W = sum(w)
    h = min(K, split * K // 3)
    u = unroll if mapping != "wide" else {0: 0, 8: 8, 16: 16, 32: 4}[unroll]
    fl = ops.tuning_flags(mapping=mapping, unroll=u)
    Xd = torch.from_numpy(X).to(dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    Xb = ops.to_blocked(Xd, 1024) if layout == "blocked" else None

    def call(k0, k1, acc, fin):
        kw = dict(acc_in=acc, W=W if fin else None, flags=fl)
        if layout == "strided":
            ops.reduce_slab(Xd[k0:k1], w32[k0:k1].contiguous(), out, **kw)
        elif layout == "rows":
            ops.reduce_rows([Xd[k] for k in range(k0, k1)], w32[k0:k1].contiguous(), out, **kw)
        else:
            ops.reduce_blocked(Xb, w32[k0:k1].contiguous(), out, B=k1 - k0, r0=k0, **kw)

    if h:
        call(0, h, None, False)
        call(h, K, out, True)
    else:
        call(0, K, None, True)
    same(out.cpu().numpy(), ref.reduce(X, w, W=W))


class _TwoParams(torch.nn.Module):
    """A client model whose flat vector is one client row (two ragged
    parameter tensors, so the pack walks a segment boundary)."""

    def __init__(self, P, dev):
        super().__init__()
        a = max(1, P // 3)
        self.a = torch.nn.Parameter(torch.empty(a, device=dev))
        self.b = torch.nn.Parameter(torch.empty(P - a, device=dev)) if P > a else None

    def load(self, row):
        with torch.no_grad():
            self.a.copy_(row[: self.a.numel()])
            if self.b is not None:
                self.b.copy_(row[self.a.numel():])


@SETTINGS
@given(rounds(max_k=20, max_p=4000), st.integers(1, 7), st.booleans(),
       st.lists(st.integers(0, 4), min_size=20, max_size=20),
       st.sampled_from(["pop", "fedavg", "adabest"]))
def test_mixed_sources_random_stream(dev, r, max_rows, borrow, kinds, final):
    """Every way a client vector reaches the aggregator, interleaved at
    random in one round: pageable host and pinned host (overwritten right
    after add) into the host key "h"; HBM (borrowed or packed), a model
    vectorized into a reserved slab row, and a reservation whose client never
    arrives into the HIP key "p" (one key holds one device, as the
    reference's running sum does; an add across them raises, checked once);
    a mid-stream get; then pop or the fused pop + server step.  Bitwise vs
    the oracle."""
    from fedsim_amd import ops
    from fedsim_amd.utils import SerialAggregator, vectorize_module

    X, w = r
    K, P = X.shape
    agg = SerialAggregator(max_rows=max_rows, borrow=borrow)
    model = _TwoParams(P, dev)
    pinned = torch.empty(P).pin_memory()
    on_host = []
    for k in range(K):
        kind = kinds[k]
        if kind == 4:
            agg.reserve("p", P, dev)  # a client that diverges after its reservation
            kind = k % 4
        if kind == 0:
            src = torch.from_numpy(X[k].copy())
        elif kind == 1:
            pinned.copy_(torch.from_numpy(X[k]))
            src = pinned
        elif kind == 2:
            src = torch.from_numpy(X[k].copy()).to(dev)
        else:
            model.load(torch.from_numpy(X[k]).to(dev))
            src = vectorize_module(model, out=agg.reserve("p", P, dev))
        on_host.append(kind in (0, 1))
        key = "h" if on_host[-1] else "p"
        other = "p" if on_host[-1] else "h"
        if k == K // 2 and other in agg:  # once per round: the other key refuses it
            with pytest.raises(RuntimeError, match="same device"):
                agg.add(other, src, w[k])
        agg.add(key, src, w[k])
        if kind == 1:
            pinned.fill_(float("nan"))
        if k == K // 2:
            for kk, host in (("h", True), ("p", False)):
                sel = [i for i in range(k + 1) if on_host[i] == host]
                if sel:
                    ws = [w[i] for i in sel]
                    same(agg.get(kk).cpu().numpy(), ref.reduce(X[sel], ws, W=sum(ws) or None))
    if K == 0:
        assert "p" not in agg and "h" not in agg
        return
    hsel = [i for i in range(K) if on_host[i]]
    if hsel:
        ws = [w[i] for i in hsel]
        got = agg.pop("h")
        assert got.device.type == "cpu"
        same(got.numpy(), ref.reduce(X[hsel], ws, W=sum(ws) or None))
    dsel = [i for i in range(K) if not on_host[i]]
    if not dsel:
        assert "p" not in agg
        return
    X, w = X[dsel], [w[i] for i in dsel]
    W = sum(w)
    avg = ref.reduce(X, w, W=W if W else None)
    if final == "pop":
        same(agg.pop("p").cpu().numpy(), avg)
        return
    cloud0 = np.random.default_rng(K * 7 + P).normal(0, 0.05, P).astype(np.float32)
    aux0 = np.random.default_rng(P).normal(0, 0.05, P).astype(np.float32)
    st_ = ref.ServerState(final, cloud0, dict(lr=0.3, momentum=0.9),
                          aux=aux0 if final == "adabest" else None, coef=0.6)
    st_.step(avg)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    aux = torch.from_numpy(aux0.copy()).to(dev) if final == "adabest" else None
    buf = torch.empty_like(cloud)
    agg.pop_step("p", ops.ServerStep(final, cloud, lr=0.3, momentum=0.9, coef=0.6, aux=aux,
                                     momentum_buf=buf, momentum_init=True))
    same(cloud.cpu().numpy(), st_.cloud)
    same(buf.cpu().numpy(), st_.buf)


@st.composite
def ref_rounds(draw):
    """A bf16 / fp16 / fp64 key: K rows of P values (normal, huge, tiny,
    signed zeros, infinities), Python int / float weights (negative and zero
    included), and a max_rows that drains in pieces."""
    dtype = draw(st.sampled_from(["bfloat16", "float16", "float64"]))
    K = draw(st.integers(1, 24))
    P = draw(st.integers(1, 3000))
    scale = draw(st.sampled_from([1e-3, 1.0, 300.0, 6e4]))
    special = draw(st.booleans())
    seed = draw(st.integers(0, 2 ** 31 - 1))
    w = draw(st.lists(st.one_of(st.integers(-50, 600), st.floats(-4.0, 4.0, width=32)),
                      min_size=K, max_size=K))
    max_rows = draw(st.integers(1, 30))
    return dtype, K, P, scale, special, seed, w, max_rows


@SETTINGS
@given(ref_rounds())
def test_generic_kernel_matches_reference_arithmetic(dev, case):
    """fedagg_reduce_rows_ref through the drop-in (HIP values, drained every
    max_rows rows) against the reference's own CPU arithmetic on the same
    values: bit for bit, NaNs compared as NaN (inf * 0, inf - inf: their bits
    are not pinned even within ATen -- its scalar bf16 conversion writes
    0x7FC0, its AVX-512 one 0xFFFF)."""
    from fedsim_amd.utils import SerialAggregator
    from oracle.reference_loop import ReferenceSerialAggregator

    dtype, K, P, scale, special, seed, w, max_rows = case
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(K, P, generator=g, dtype=torch.float64) * scale
    if special:
        idx = torch.randint(0, K * P, (max(1, K * P // 50),), generator=g)
        vals = torch.tensor([0.0, -0.0, float("inf"), -float("inf"), 1e-42, 7e4])
        X.view(-1)[idx] = vals[torch.randint(0, len(vals), idx.shape, generator=g)].double()
    X = X.to(dt)
    agg, ref_agg = SerialAggregator(max_rows=max_rows), ReferenceSerialAggregator()
    for k in range(K):
        agg.add("p", X[k].to(dev), w[k])
        ref_agg.add("p", X[k], w[k])
    for got, exp in ((agg.get_sum("p"), ref_agg.get_sum("p")), (agg.pop("p"), ref_agg.pop("p"))):
        got = got.cpu()
        assert got.dtype == exp.dtype and got.shape == exp.shape
        nan_g, nan_e = torch.isnan(got), torch.isnan(exp)
        assert torch.equal(nan_g, nan_e)
        ib = torch.int64 if dt == torch.float64 else torch.int16
        assert torch.equal(got[~nan_g].view(ib), exp[~nan_e].view(ib))


# The tile ladders of k_reduce_rows_ref (fedagg_kernels.hip launch_rows_ref
# and fedagg_reduce_rows_f32): P ranges that select each tile.
_REF_RUNGS = {
    "bfloat16": [(1, 4_100_000), (4_190_000, 8_300_000), (8_380_000, 9_000_000)],
    "float16": [(1, 4_100_000), (4_190_000, 8_300_000), (8_380_000, 9_000_000)],
    "float64": [(1, 1_000_000), (1_050_000, 3_100_000), (3_150_000, 3_600_000)],
}
WIDE = settings(max_examples=24, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow,
                                       HealthCheck.function_scoped_fixture])


@st.composite
def wide_ref_rounds(draw):
    dtype = draw(st.sampled_from(sorted(_REF_RUNGS)))
    lo, hi = draw(st.sampled_from(_REF_RUNGS[dtype]))
    P = draw(st.integers(lo, hi))
    K = draw(st.integers(1, 8))
    w = draw(st.lists(st.one_of(st.integers(-50, 600), st.floats(-4.0, 4.0, width=32),
                                st.sampled_from([0.37, 0.1, 1.7])), min_size=K, max_size=K))
    split = draw(st.integers(0, K))  # rows before the acc_in continuation
    off = draw(st.one_of(st.none(), st.integers(0, K - 1)))  # a row off 16-B alignment
    seed = draw(st.integers(0, 2 ** 31 - 1))
    return dtype, P, K, w, split, off, seed


@WIDE
@given(wide_ref_rounds())
def test_generic_kernel_tiles_random(dev, case):
    """fedagg_reduce_rows_ref at random sizes around every tile of the ladder,
    vector or all-scalar path, one call or a running sum continued with
    acc_in: bitwise the reference's CPU arithmetic (finite inputs)."""
    from fedsim_amd import ops
    from oracle.reference_loop import ReferenceSerialAggregator

    dtype, P, K, w, split, off, seed = case
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(seed)
    X = [(torch.randn(P, generator=g, dtype=torch.float32) * 0.5).to(dt) for _ in range(K)]
    ref = ReferenceSerialAggregator()
    for k in range(K):
        ref.add("p", X[k], w[k])
    want = ref.get_sum("p")
    rows = [x.to(dev) for x in X]
    if off is not None:
        big = torch.empty(P + 1, dtype=dt, device=dev)
        big[1:].copy_(X[off])
        rows[off] = big[1:]
    out = torch.empty(P, dtype=dt, device=dev)
    if 0 < split < K:
        head = torch.empty(P, dtype=dt, device=dev)
        ops.reduce_rows_ref(rows[:split], w[:split], head)
        ops.reduce_rows_ref(rows[split:], w[split:], out, acc_in=head)
    else:
        ops.reduce_rows_ref(rows, w, out)
    got = out.cpu()
    nan_g, nan_e = torch.isnan(got), torch.isnan(want)
    assert torch.equal(nan_g, nan_e)
    ib = torch.int64 if dt == torch.float64 else torch.int16
    assert torch.equal(got[~nan_g].view(ib), want[~nan_e].view(ib))


@WIDE
@given(st.integers(1_500_000, 5_000_000), st.integers(1, 20), st.booleans(),
       st.integers(0, 20), st.integers(0, 2 ** 31 - 1))
def test_fp32_tile_rows_random(dev, P, K, finalize, split, seed):
    """fedagg_reduce_rows_f32 on borrowed rows at random sizes around its tile
    thresholds (P % 4 != 0 keeps the narrow kernels): bitwise the narrow
    kernels (mapping forced), with the divide and an acc_in continuation."""
    from fedsim_amd import ops

    g = torch.Generator(device=dev).manual_seed(seed)
    rows = [torch.empty(P, device=dev).normal_(0, 1, generator=g) for _ in range(K)]
    wl = [float(v) for v in torch.randint(-5, 600, (K,), generator=torch.Generator().manual_seed(seed))]
    wl[0] = 0.37
    w32 = torch.tensor([ops.fl32(x) for x in wl], dtype=torch.float32, device=dev)
    W = sum(wl) if finalize and sum(wl) != 0 else None
    split = min(split, K)
    outs = []
    for flags in (0, 3 << 18):  # default mapping (tiles where they apply); FEDAGG_MAP VW=2
        out = torch.empty(P, device=dev)
        if 0 < split < K:
            acc = torch.empty(P, device=dev)
            ops.reduce_rows(rows[:split], w32[:split], acc, flags=flags)
            ops.reduce_rows(rows[split:], w32[split:], out, acc_in=acc, W=W, flags=flags)
        else:
            ops.reduce_rows(rows, w32, out, W=W, flags=flags)
        outs.append(out)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
