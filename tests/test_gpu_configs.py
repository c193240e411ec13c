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
  (d) configs 1-3 at the CLI's default participation (-c 0.01): config 1
      (FedAvg, SimpleMLP, 500 clients -> K=5, pageable host client vectors,
      cloud on the host, as ``fed-learn --device cpu`` runs it) and configs 2
      and 3 (FedAvg / AdaBest mu 0.01 beta 0.6, SimpleCNN2(num_classes=100),
      1000 clients -> K=10, host and HBM) through CentralFLAlgorithm for 3
      rounds: bitwise the reference's own round loop (tests/golden/
      configs.json, tools/gen_golden_configs.py)
  (e) configs 2 and 3 at full participation (-c 1.0): 1000 GPU clients of
      SimpleCNN2's size (1 085 668) writing their vectors into the round's
      slab rows (the production client path, local_updates.sgd_update),
      through CentralFLAlgorithm -> FedAvg.optimize / AdaBest.optimize (the
      split pop + server step that ops.fuse_step_pays picks at this size):
      bitwise against the oracle on 4 096 + 128 sampled columns

Reference arithmetic: SerialAggregator.add / pop (fedsim/utils/aggregators.py
:17-40, 104-122), FedAvg.optimize (training/fedavg.py:193-208), AdaBest.optimize
(training/adabest.py:172-189).
"""
import json
import os
import random
from functools import partial

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DIR, bits
from oracle import ref
from oracle import synthetic_fl as S
from oracle import vectors as V

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



with open(os.path.join(GOLDEN_DIR, "configs.json")) as _f:
    _CFG = json.load(_f)


@pytest.mark.parametrize("device", ["cpu", "cuda"])
@pytest.mark.parametrize("rid", [r["id"] for r in _CFG["runs"]])
def test_configs_1_to_3_cli_defaults_bitwise_vs_reference_round_loop(rid, device):
    """(d) The reference's own 3-round trajectory of the config at the CLI's
    default participation, bit for bit: device="cpu" gives pageable host
    client vectors and a host cloud (the ingest path), device="cuda" HBM
    ones (borrowed rows)."""
    from fedsim_amd import models
    from fedsim_amd.distributed.centralized import training

    run = [r for r in _CFG["runs"] if r["id"] == rid][0]
    cls = S.make_algorithm(getattr(training, run["algorithm"]))
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(data_manager=S.FakeDataManager(run["num_clients"]), metric_logger=None,
              num_clients=run["num_clients"], sample_scheme="uniform",
              sample_rate=run["sample_rate"],
              model_def=partial(getattr(models, run["model"]), **run["model_kwargs"]), epochs=1,
              criterion_def="CrossEntropyScore", optimizer_def=partial(torch.optim.SGD, lr=1.0),
              device=device, **run["alg_kwargs"])
    scores = alg.train(rounds=_CFG["rounds"])
    st = alg.get_server_storage()
    cloud = st.read("cloud_params")
    assert cloud.device.type == device and cloud.numel() == run["P"]
    assert V.sha256(cloud.detach().cpu().numpy()) == run["cloud_sha256"]
    if "avg_params_sha256" in run:
        assert V.sha256(st.read("avg_params").detach().cpu().numpy()) == run["avg_params_sha256"]
    assert {k: float(v) for k, v in scores.items()} == run["scores"]


def _gpu_slab_client(record, cols, slab_row=True):
    """A client that trains on the GPU, as local_updates.sgd_update hands its
    update over: its model's parameters become views of one fresh device
    vector (cloud + a seeded N(0, 1e-3) delta), which vectorize_module packs
    into the round's reserved slab row (``slab_row=False``: a fresh
    ``torch.cat`` vector instead, the reference client's own hand-over, which
    the aggregator borrows in place).  Records (vector[cols], weight)."""
    from torch.nn.utils import parameters_to_vector, vector_to_parameters

    from fedsim_amd.utils import hand_over, vectorize_module
    from fedsim_amd.utils.slab_rows import reserve_round_row

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        model = ctx["model"]
        base = parameters_to_vector(model.parameters()).detach()
        g = torch.Generator(device=base.device).manual_seed(1_000_003 * rounds + id)
        local = base + torch.empty_like(base).normal_(0.0, 1e-3, generator=g)
        vector_to_parameters(local, model.parameters())
        row = None
        if slab_row:
            row = reserve_round_row("local_params", model)
            assert row is not None and row.in_slab
        n = len(datasets[train_split_name])
        record.append((local[cols], n))
        # a fresh vector the client keeps nowhere: declared handed over, so
        # the round driver's aggregator reads it where it lies (borrowed)
        return dict(local_params=hand_over(vectorize_module(model, out=row)),
                    num_steps=max(1, n // 32),
                    diverged=False, num_samples={train_split_name: n},
                    metrics={train_split_name: {"loss": 1.0 + 0.001 * id}})

    return send_to_server


@pytest.mark.parametrize("slab_row", [True, False], ids=["slab_rows", "borrowed"])
@pytest.mark.parametrize("algo", ["FedAvg", "AdaBest", "FedNova"])
def test_configs_2_3_full_participation_1000x1_085_668(algo, slab_row):
    """(e) -c 1.0: K = 1000 clients x SimpleCNN2's 1 085 668 parameters, one
    round through the round driver with every client in a slab row, or
    handing over a fresh vector that the aggregator borrows (the row-pointer
    kernels); the server step is the split pass at this size."""
    from fedsim_amd import models, ops
    from fedsim_amd.distributed.centralized import training

    _need(10)
    n_clients, P = 1000, 1_085_668
    cols = _sample_cols(P)
    c = torch.from_numpy(cols).to(DEV)
    record = []
    base = getattr(training, algo)
    cls = type("Gpu" + algo, (base,), {"send_to_server": _gpu_slab_client(record, c, slab_row)})
    akw = dict(mu=0.01, beta=0.6) if algo == "AdaBest" else {}
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(data_manager=S.FakeDataManager(n_clients), metric_logger=None,
              num_clients=n_clients, sample_scheme="uniform", sample_rate=1.0,
              model_def=partial(models.SimpleCNN2, num_classes=100), epochs=1,
              criterion_def="CrossEntropyScore", optimizer_def=partial(torch.optim.SGD, lr=1.0),
              device="cuda", **akw)
    st = alg.get_server_storage()
    cloud0 = st.read("cloud_params").detach()[c].cpu().numpy()
    prev0 = st.read("avg_params")[c].cpu().numpy() if algo == "AdaBest" else None
    assert st.read("cloud_params").numel() == P
    split, borrowed = [], []

    def spy(*a, **k):
        borrowed.append(bool(k.get("borrowed", False)))
        split.append(not orig(*a, **k))
        return orig(*a, **k)

    orig = ops.fuse_step_pays
    ops.fuse_step_pays = spy
    try:
        alg.train(rounds=0)  # one round
    finally:
        ops.fuse_step_pays = orig
    assert len(record) == n_clients
    assert split and all(split)  # the split pop + step at this size
    assert borrowed == [not slab_row]  # rows read in the slab, or where the clients left them
    sub = torch.stack([v for v, _ in record]).cpu().numpy()  # [K, n] in arrival order
    # FedAvg: n_train (int); AdaBest: 1; FedNova: n_train / num_steps (float,
    # fednova.py:58-59; the client sends num_steps = max(1, n // 32))
    w = {"FedAvg": [n for _, n in record], "AdaBest": [1] * n_clients,
         "FedNova": [n / max(1, n // 32) for _, n in record]}[algo]
    avg = ref.reduce(sub, w, W=sum(w))
    if algo in ("FedAvg", "FedNova"):
        state = ref.ServerState("fedavg", cloud0, dict(lr=1.0))
    else:
        state = ref.ServerState("adabest", cloud0, dict(lr=1.0), aux=prev0, coef=0.6)
    state.step(avg)
    cloud = st.read("cloud_params").detach()
    np.testing.assert_array_equal(bits(cloud[c].cpu().numpy()), bits(state.cloud))
    if algo == "AdaBest":
        np.testing.assert_array_equal(bits(st.read("avg_params")[c].cpu().numpy()), bits(avg))
    assert torch.isfinite(cloud).all()
