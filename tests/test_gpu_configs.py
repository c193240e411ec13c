"""GPU parity at the BASELINE configs' own workloads (the sizes bench.py times),
against the oracle on sampled columns -- 4096 random ones plus the first and
last 64 (the ragged column block) -- and through size-independent properties.

  (a) the headline round: fedagg_reduce_step_blocked_f32 (reduce + divide +
      server step in one pass) at K=1000 x P=25 M, C=4096, exactly as
      bench.py's default line runs it; FedAvg lr 1.0 and AdaBest beta 0.6
  (b) config 4's per-rank shard: rank 7 of 8 of a 10 000 x 25 M model,
      10 000 x 3 124 608 columns (125 GB), through sharding.param_sharded_step
  (c) config 5's streamed pool pass: a resident 200-row pool at P = 125 M
      re-read for 4 passes (700 clients) chained through acc_in, bitwise in
      order; and the client-sharded (reordered) decomposition of the same
      clients over 8 virtual ranks: normwise <= 1e-6 vs the in-order result
      and the gamma_K forward-error bound vs fp64 on the sampled columns

Reference arithmetic: SerialAggregator.add / pop (fedsim/utils/aggregators.py
:17-40, 104-122), FedAvg.optimize (training/fedavg.py:193-208), AdaBest.optimize
(training/adabest.py:172-189).
"""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _need(gb):
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(DEV)
    if free < gb * 1e9:
        pytest.skip(f"needs {gb} GB of free HBM, {free / 1e9:.0f} free")


def _sample_cols(P, n=4096, seed=3):
    rng = np.random.default_rng(seed)
    cols = np.concatenate([np.arange(64), rng.choice(P, size=n, replace=False),
                           np.arange(P - 64, P)])
    return np.unique(cols)


def _blocked_cols(Xb, cols, rows=None):
    """[len(cols), B] -> numpy [B, len(cols)] of a column-blocked slab."""
    C = Xb.shape[2]
    c = torch.from_numpy(cols).to(DEV)
    sub = Xb[c // C, :, c % C]  # [n, Kcap]
    if rows is not None:
        sub = sub[:, rows[0]:rows[1]]
    return np.ascontiguousarray(sub.t().cpu().numpy())


def _fill_realistic(Xb, seed):
    """base ~ N(0, 0.05) per column + N(0, 1e-3) per element (bench.py's
    synthetic client vectors: non-cancelling sums)."""
    nb, K, C = Xb.shape
    g = torch.Generator(device=DEV).manual_seed(seed)
    base = torch.empty((nb, 1, C), device=DEV).normal_(0.0, 0.05, generator=g)
    for b0 in range(0, nb, 128):
        blk = Xb[b0:b0 + 128]
        blk.normal_(0.0, 1e-3, generator=g).add_(base[b0:b0 + 128])
    return Xb


def _weights(K, seed=11):
    return [int(v) for v in np.random.default_rng(seed).integers(50, 601, size=K)]


def _w32(w):
    from fedsim_amd import ops

    return torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=DEV)


def test_headline_round_fused_step_1000x25M():
    """(a) bench.py's default line: the same kernel on the same shape."""
    from fedsim_amd import ops

    _need(110)
    K, P, C = 1000, 25_000_000, 4096
    Xb = _fill_realistic(torch.empty(ops.blocked_shape(K, P, C), device=DEV), 17)
    w = _weights(K)
    W = sum(w)
    w32 = _w32(w)
    cols = _sample_cols(P)
    sub = _blocked_cols(Xb, cols)
    avg_ref = ref.reduce(sub, w, W=W)
    rng = np.random.default_rng(4)
    cloud0 = rng.normal(0, 0.05, size=P).astype(np.float32)
    prev0 = rng.normal(0, 0.05, size=P).astype(np.float32)
    assert ops.column_mapping(P, 0, B=K) == ("narrow2", 8)  # the bench's instance

    # FedAvg, lr 1.0 (FedAvg.optimize's default server SGD), pseudo-gradient stored
    cloud = torch.from_numpy(cloud0).to(DEV)
    grad = torch.empty_like(cloud)
    ops.reduce_blocked_step(Xb, w32, ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad),
                            W=W)
    st = ref.ServerState("fedavg", cloud0[cols], dict(lr=1.0))
    st.step(avg_ref)
    np.testing.assert_array_equal(bits(cloud[torch.from_numpy(cols).to(DEV)].cpu().numpy()),
                                  bits(st.cloud))
    np.testing.assert_array_equal(bits(grad[torch.from_numpy(cols).to(DEV)].cpu().numpy()),
                                  bits(st.grad))
    # the column sums are finite and every column was written
    assert torch.isfinite(cloud).all() and torch.isfinite(grad).all()

    # AdaBest beta 0.6 (config 3's rule) on the same rows, weights 1
    ones = [1] * K
    avg1 = ref.reduce(sub, ones, W=K)
    cloud = torch.from_numpy(cloud0).to(DEV)
    prev = torch.from_numpy(prev0).to(DEV)
    ops.reduce_blocked_step(Xb, _w32(ones),
                            ops.ServerStep("adabest", cloud, lr=1.0, coef=0.6, aux=prev), W=K)
    st = ref.ServerState("adabest", cloud0[cols], dict(lr=1.0), aux=prev0[cols], coef=0.6)
    st.step(avg1)
    c = torch.from_numpy(cols).to(DEV)
    np.testing.assert_array_equal(bits(cloud[c].cpu().numpy()), bits(st.cloud))
    np.testing.assert_array_equal(bits(prev[c].cpu().numpy()), bits(st.aux))


def test_config4_rank_shard_10000x3_125M():
    """(b) the last rank's shard of config 4 through the library call a
    parameter-sharded rank makes (sharding.param_sharded_step)."""
    from fedsim_amd import ops, sharding

    _need(135)
    K, Pfull, world, rank = 10_000, 25_000_000, 8, 7
    lo, hi = sharding.shard_span(Pfull, rank, world)
    P = hi - lo
    assert P == 3_124_608 and hi == Pfull
    C = ops.choose_block_cols(P)
    Xb = _fill_realistic(torch.empty(ops.blocked_shape(K, P, C), device=DEV), 23)
    w = _weights(K, seed=12)
    W = sum(w)
    cols = _sample_cols(P)
    sub = _blocked_cols(Xb, cols)
    cloud0 = np.random.default_rng(5).normal(0, 0.05, size=P).astype(np.float32)
    cloud = torch.from_numpy(cloud0).to(DEV)
    grad = torch.empty_like(cloud)
    sharding.param_sharded_step(Xb, _w32(w), W, ops.ServerStep("fedavg", cloud, lr=1.0,
                                                               grad_out=grad))
    st = ref.ServerState("fedavg", cloud0[cols], dict(lr=1.0))
    st.step(ref.reduce(sub, w, W=W))
    c = torch.from_numpy(cols).to(DEV)
    np.testing.assert_array_equal(bits(cloud[c].cpu().numpy()), bits(st.cloud))
    np.testing.assert_array_equal(bits(grad[c].cpu().numpy()), bits(st.grad))
    # property: the fused shard pass == reduce + stored-average step (split)
    cloud2 = torch.from_numpy(cloud0).to(DEV)
    avg = torch.empty(P, device=DEV)
    ops.reduce_blocked(Xb, _w32(w), avg, W=W, flags=ops.default_flags(C))
    ops.ServerStep("fedavg", cloud2, lr=1.0).apply(avg)
    assert torch.equal(cloud.view(torch.int32), cloud2.view(torch.int32))


def test_config5_streamed_pool_and_reordered_decomposition():
    """(c) config 5's per-GPU pass structure at P = 125 M."""
    from fedsim_amd import ops

    _need(110)
    R, P = 200, 125_000_000
    counts = [200, 200, 200, 100]  # 700 clients streamed from the 200-row pool
    K = sum(counts)
    C = ops.choose_block_cols(P)
    pool = _fill_realistic(torch.empty(ops.blocked_shape(R, P, C), device=DEV), 29)
    w = _weights(K, seed=13)
    W = sum(w)
    w32 = _w32(w)
    flags = ops.default_flags(C)
    acc = torch.empty(P, device=DEV)
    k0 = 0
    for i, n in enumerate(counts):
        ops.reduce_blocked(pool, w32[k0:k0 + n], acc, B=n, acc_in=None if i == 0 else acc,
                           W=W if i == len(counts) - 1 else None, flags=flags)
        k0 += n
    cols = _sample_cols(P)
    sub = _blocked_cols(pool, cols)  # [R, n]
    rows = np.concatenate([sub[:n] for n in counts])  # the client sequence
    exp = ref.reduce(rows, w, W=W)
    c = torch.from_numpy(cols).to(DEV)
    np.testing.assert_array_equal(bits(acc[c].cpu().numpy()), bits(exp))

    # client-sharded decomposition (what 8 ranks + all-reduce compute): each
    # virtual rank sums its contiguous run of the sequence from zero, the
    # partials are summed in rank order, then one divide by fl32(W)
    world = 8
    offs = np.cumsum([0] + counts)  # clients [offs[i], offs[i+1]) = pool rows [0, n_i)
    bounds = [K * r // world for r in range(world + 1)]
    total = torch.zeros(P, device=DEV)
    part = torch.empty(P, device=DEV)
    for r in range(world):
        a, b = bounds[r], bounds[r + 1]
        first = True
        for i, n in enumerate(counts):
            s, e = max(a, offs[i]), min(b, offs[i] + n)
            if s >= e:
                continue
            ops.reduce_blocked(pool, w32[s:e], part, B=int(e - s), r0=int(s - offs[i]),
                               acc_in=None if first else part, flags=flags)
            first = False
        total.add_(part)
    reord = ops.finalize(total, W)
    rel = float(torch.linalg.vector_norm((reord - acc).double()) /
                torch.linalg.vector_norm(acc.double()))
    assert rel <= 1e-6, rel
    # gamma_K forward-error bound against fp64 on the sampled columns
    x64 = rows.astype(np.float64)
    w64 = np.array([np.float32(v) for v in w], dtype=np.float64)
    y64 = (w64[:, None] * x64).sum(0) / np.float64(np.float32(W))
    gamma = K * 2.0 ** -24 / (1 - K * 2.0 ** -24)
    bound = gamma * np.abs(w64[:, None] * x64).sum(0) / np.float32(W) + np.abs(y64) * 2.0 ** -23
    got = reord[c].cpu().numpy().astype(np.float64)
    assert np.all(np.abs(got - y64) <= bound)

