"""FEDAGG_FAST: the reordered split-K reduction for small P (include/fedagg.h).
Not the reference's summation order, so the bar is the normwise one SURVEY
§8c sets for reordered sums — ||y - y_ref|| <= 1e-6 ||y_ref|| against the
bit-exact oracle, and elementwise |y - y64| <= gamma_K * sum|w_k x_k| / W
against an fp64 reduction — plus run-to-run determinism, and bitwise equality
with the exact kernels wherever the mode adds no parallelism (large P)."""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def _check_normwise(got, X, w, W, cancelling=False):
    """Against the fp64 value y64: the elementwise gamma_K forward-error bound,
    and no further from y64 than the reference's own sequential fp32 sum is
    (x2; that sum carries ~sqrt(K) u of error itself, so at K = 9000 the two
    fp32 results can differ by more than 1e-6 while both are correct).  For
    realistic client vectors (base + small per-client noise) at
    K <= 1000, also normwise 1e-6 against the reference's (bit-exact oracle)
    result, the §8c bar."""
    want = ref.reduce(X, w, W=W).astype(np.float64)
    w32 = np.array([np.float32(v) for v in w], dtype=np.float64)
    y64 = (w32[:, None] * X.astype(np.float64)).sum(0) / np.float64(np.float32(W))
    g = got.astype(np.float64)
    assert np.linalg.norm(g - y64) <= 2 * np.linalg.norm(want - y64) + 1e-30
    if not cancelling and X.shape[0] <= 1000:
        assert np.linalg.norm(g - want) <= 1e-6 * np.linalg.norm(want)
    K = X.shape[0]
    u = 2.0 ** -24
    gamma = (K + 2) * u / (1 - (K + 2) * u)
    bound = gamma * (np.abs(w32[:, None] * X.astype(np.float64)).sum(0)) / np.float32(W)
    assert np.all(np.abs(got.astype(np.float64) - y64) <= bound + 1e-45)


@pytest.mark.parametrize("dist", ["realistic", "normal"])
@pytest.mark.parametrize("layout", ["strided", "rows", "blocked"])
@pytest.mark.parametrize("K,P", [(1, 5), (37, 1), (300, 7_850), (1000, 1_023), (4100, 333),
                                 (9000, 4_099)])
def test_fast_reduce_normwise_and_deterministic(K, P, layout, dist, dev):
    from fedsim_amd import ops

    X = V.client_rows(dist, K, P, 7 + K)
    w = V.client_weights("fedavg", K, 7 + K)
    W = sum(w)
    Xd = torch.from_numpy(X).to(dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    fl = ops.tuning_flags(fast=True)
    outs = []
    for _ in range(2):
        out = torch.empty(P, dtype=torch.float32, device=dev)
        h = K // 3  # two chained batches: acc_in is folded in after the partials
        if layout == "strided":
            ops.reduce_slab(Xd[:h], w32[:h], out, flags=fl) if h else out.zero_()
            ops.reduce_slab(Xd[h:], w32[h:].contiguous(), out, acc_in=out, W=W, flags=fl)
        elif layout == "rows":
            rows = [Xd[k] for k in range(K)]
            ops.reduce_rows(rows[:h], w32[:h], out, flags=fl) if h else out.zero_()
            ops.reduce_rows(rows[h:], w32[h:].contiguous(), out, acc_in=out, W=W, flags=fl)
        else:
            Xb = ops.to_blocked(Xd, 1024)
            ops.reduce_blocked(Xb, w32[:h], out, B=h, flags=fl) if h else out.zero_()
            ops.reduce_blocked(Xb, w32[h:].contiguous(), out, B=K - h, acc_in=out, W=W, flags=fl,
                               r0=h)
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(bits(outs[0]), bits(outs[1]))
    _check_normwise(outs[0], X, w, W, cancelling=(dist == "normal"))


def test_fast_is_exact_where_it_adds_nothing(dev):
    """At P >= 65,536 one column per lane already fills the chip: the flag falls
    back to the exact kernels, bit for bit."""
    from fedsim_amd import ops

    K, P = 5, 70_000
    X = V.client_rows("realistic", K, P, 3)
    w = V.client_weights("fedavg", K, 3)
    Xd = torch.from_numpy(X).to(dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    ops.reduce_slab(Xd, w32, out, W=sum(w), flags=ops.tuning_flags(fast=True))
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.reduce(X, w, W=sum(w))))


@pytest.mark.parametrize("borrow", [False, True])
@pytest.mark.parametrize("algo", ["fedavg", "adabest", "feddyn"])
def test_fast_aggregator_pop_step(algo, borrow, dev):
    """SerialAggregator(fast=True): the ring drains and the fused server step
    take the split-K kernels; the step matches the oracle's step applied to
    the fast average bit for bit, and the average matches normwise."""
    from fedsim_amd import ops
    from fedsim_amd.utils import SerialAggregator

    K, P = 700, 7_850
    X = V.client_rows("realistic", K, P, 11)
    w = V.client_weights("fedavg", K, 11)
    W = sum(w)
    agg = SerialAggregator(fast=True, borrow=borrow, max_rows=256)
    avg_agg = SerialAggregator(fast=True, borrow=borrow, max_rows=256)
    for k in range(K):
        row = torch.from_numpy(X[k].copy()).to(dev)
        agg.add("p", row, w[k])
        avg_agg.add("p", row.clone(), w[k])
    avg = avg_agg.pop("p").cpu().numpy()
    _check_normwise(avg, X, w, W)
    cloud0 = V.cloud_vector(P, 12)
    aux0 = V.cloud_vector(P, 13)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    aux = torch.from_numpy(aux0.copy()).to(dev)
    step = ops.ServerStep(algo, cloud, lr=0.7, coef=0.6, aux=None if algo == "fedavg" else aux)
    agg.pop_step("p", step)
    want = ref.ServerState(algo, cloud0, dict(lr=0.7), coef=0.6,
                           aux=None if algo == "fedavg" else aux0)
    want.step(avg)
    np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(want.cloud))
