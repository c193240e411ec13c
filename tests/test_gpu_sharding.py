"""The multi-GPU protocols of fedsim_amd.sharding with the real HIP per-rank
reducer, on a one-rank RCCL ("nccl") process group (the 8-GPU run belongs to the
driver).  Bit-exact vs the oracle for param / chain; the all-reduce path must
still be exact at one rank (nothing is reordered)."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu


def _file_store(d):
    """A file rendezvous for the spawned gloo ranks: no TCP port to race
    for (a port picked free and then bound by the store can be taken in
    between: EADDRINUSE on a shared box, r05ae)."""
    return "file://" + os.path.join(d, "pg_store")


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist

    if dist.is_initialized():
        yield dist
        return
    d = tempfile.mkdtemp()
    dist.init_process_group("nccl", init_method=_file_store(d), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()
    shutil.rmtree(d, ignore_errors=True)


@pytest.mark.parametrize("mode", ["param", "chain", "allreduce"])
def test_sharding_protocols_one_rank(mode, pg):
    from fedsim_amd import sharding

    dev = torch.device("cuda", 0)
    K, P = 37, 100_003
    X = V.client_rows("normal", K, P, 9)
    w = V.client_weights("fedavg", K, 9)
    W = sum(w)
    exp = ref.reduce(X, w, W=W)
    Xd = torch.from_numpy(X).to(dev)
    w32 = sharding.weights_fp32(w, dev)
    out = torch.empty(P, device=dev)
    if mode == "param":
        lo, hi = sharding.shard_range(P, 0, 1, sharding.ALIGN)
        sharding.param_sharded(Xd[:, lo:hi], w32, W, out[lo:hi])
    elif mode == "chain":
        sharding.client_sharded_chain(Xd, w32, W, out, n_blocks=5)
    else:
        sharding.client_sharded_allreduce(Xd, w32, W, out)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(exp))


# ---------------------------------------------------------------------------
# ShardedSerialAggregator (the plugin-surface multi-GPU aggregator)
# ---------------------------------------------------------------------------
def _golden_runs():
    import json

    from conftest import GOLDEN_DIR

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        return [r for r in json.load(f)["runs"]
                if r.get("client", "synthetic") == "synthetic" and r["algorithm"] != "FedDF"]


SYN_RUNS = _golden_runs()
# client-sharded rounds refuse AdaBest: its clients' context (the running
# average_sample) depends on the earlier clients of the round
# (tests/test_sharding_gloo.py::test_client_sharded_state_divergence_and_refusal)
CS_RUNS = [r for r in SYN_RUNS if r["algorithm"] != "AdaBest"]


@pytest.fixture(scope="module")
def round_arrays():
    from conftest import GOLDEN_DIR

    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _build(run, device, factory):
    import random
    from functools import partial

    from fedsim_amd.distributed.centralized import training
    from oracle import synthetic_fl as S

    cls = S.make_algorithm(getattr(training, run["algorithm"]))
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    return cls(data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
               sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel,
               epochs=1, criterion_def="CrossEntropyScore",
               optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device=device,
               aggregator_factory=factory, **run["alg_kwargs"])


def _check_run(run, st, scores, arrays, where=""):
    for name in ("cloud_params", "avg_params", "h"):
        key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
        if key not in arrays:
            continue
        got = st.read(name, silent=True).detach().cpu().numpy()
        np.testing.assert_array_equal(bits(got), bits(arrays[key]),
                                      err_msg=f"{run['id']} {name} {where}")
    assert {k: float(v) for k, v in scores.items()} == run["scores"], run["id"]


@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("run", SYN_RUNS, ids=[f"{r['id']}-{r['algorithm']}" for r in SYN_RUNS])
def test_sharded_round_loop_one_rank_rccl(run, device, pg, round_arrays):
    """The reference's 5-round trajectories through CentralFLAlgorithm with
    the parameter-sharded aggregator on a one-rank RCCL group (HIP entries,
    borrowed HBM rows / host ingest, fused narrowed step, all-gathers)."""
    from functools import partial

    from fedsim_amd.sharding import ShardedSerialAggregator

    alg = _build(run, device, partial(ShardedSerialAggregator, borrow=True, expected_rows=5))
    scores = alg.train(rounds=4)
    _check_run(run, alg.get_server_storage(), scores, round_arrays, device)


def _gloo_gpu_worker(rank, world, store, ids, outdir):
    """One rank of a gloo group whose ranks share cuda:0 (HIP entries; the
    shards are exchanged through host memory)."""
    import json
    from functools import partial

    import torch.distributed as dist

    from fedsim_amd.sharding import ShardedSerialAggregator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        runs = {r["id"]: r for r in _golden_runs()}
        for rid in ids:
            alg = _build(runs[rid], "cuda", partial(ShardedSerialAggregator, borrow=True))
            scores = alg.train(rounds=4)
            st = alg.get_server_storage()
            out = {}
            for name in ("cloud_params", "avg_params", "h"):
                try:
                    t = st.read(name, silent=True)
                except Exception:  # noqa: BLE001 - key absent for this algorithm
                    continue
                if isinstance(t, torch.Tensor):
                    out[name] = t.detach().cpu().numpy()
            np.savez(os.path.join(outdir, f"{rid}_rank{rank}.npz"), **out)
            with open(os.path.join(outdir, f"{rid}_rank{rank}.json"), "w") as f:
                json.dump({k: float(v) for k, v in scores.items()}, f)
    finally:
        dist.destroy_process_group()


def test_sharded_round_loop_two_ranks_on_one_gpu(round_arrays):
    """Two ranks (gloo, both on cuda:0) each reduce HALF of every client
    vector with the HIP kernels and step their half of the model; after every
    round both hold the reference's full model, bit for bit."""
    import json
    import tempfile

    import torch.multiprocessing as mp

    ids = [r["id"] for r in SYN_RUNS]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_gpu_worker, args=(2, _file_store(d), ids, d), nprocs=2, join=True,
                           start_method="spawn")
        for run in SYN_RUNS:
            for r in range(2):
                got = np.load(os.path.join(d, f"{run['id']}_rank{r}.npz"))
                for name in got.files:
                    key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
                    if key in round_arrays:
                        np.testing.assert_array_equal(bits(got[name]), bits(round_arrays[key]),
                                                      err_msg=f"{run['id']} rank {r} {name}")
                with open(os.path.join(d, f"{run['id']}_rank{r}.json")) as f:
                    assert json.load(f) == run["scores"]


@pytest.mark.parametrize("borrow", [False, True])
def test_sharded_aggregator_sources_one_rank(borrow, pg):
    """Pageable and pinned host client vectors into one key and HBM-resident
    ones into another through the sharded aggregator (RCCL, one rank): get
    mid-stream, pop, and pop_step with a momentum SGD step, bitwise vs the
    oracle.  A key holds one device, as the reference's running sum does:
    a host vector added to the HIP key raises and changes nothing."""
    from fedsim_amd import ops
    from fedsim_amd.sharding import ShardedSerialAggregator

    dev = torch.device("cuda", 0)
    K, P = 29, 100_003
    X = V.client_rows("realistic", K, P, 5)
    w = V.client_weights("fedavg", K, 5)
    hk = [k for k in range(K) if k % 3 != 2]
    dk = [k for k in range(K) if k % 3 == 2]
    wh, wd = [w[k] for k in hk], [w[k] for k in dk]
    avg_h, avg_d = ref.reduce(X[hk], wh, W=sum(wh)), ref.reduce(X[dk], wd, W=sum(wd))
    for final in ("pop", "step"):
        agg = ShardedSerialAggregator(borrow=borrow)
        pinned = torch.empty(P).pin_memory()
        for k in range(K):
            if k % 3 == 0:
                src = torch.from_numpy(X[k].copy())
            elif k % 3 == 1:
                src = pinned
                src.copy_(torch.from_numpy(X[k]))
            else:
                src = torch.from_numpy(X[k].copy()).to(dev)
            agg.add("d" if k % 3 == 2 else "p", src, w[k])
            if k % 3 == 1:
                src.fill_(float("nan"))  # snapshot already taken
            if k == K // 2:
                with pytest.raises(RuntimeError, match="same device"):
                    agg.add("d", torch.from_numpy(X[k].copy()), w[k])
                sel = [i for i in hk if i <= k]
                ws = [w[i] for i in sel]
                mid = agg.get("p")
                np.testing.assert_array_equal(bits(mid.cpu().numpy()),
                                              bits(ref.reduce(X[sel], ws, W=sum(ws))))
        outd = agg.pop("d")
        assert outd.device == dev
        np.testing.assert_array_equal(bits(outd.cpu().numpy()), bits(avg_d))
        if final == "pop":
            out = agg.pop("p")
            assert out.device.type == "cpu"  # the values were host tensors
            np.testing.assert_array_equal(bits(out.numpy()), bits(avg_h))
            continue
        cloud0 = V.cloud_vector(P, 6)
        st = ref.ServerState("fedavg", cloud0, dict(lr=0.3, momentum=0.9))
        st.step(avg_h)
        cloud = torch.from_numpy(cloud0.copy()).to(dev)
        grad = torch.empty_like(cloud)
        buf = torch.empty_like(cloud)
        step = ops.ServerStep("fedavg", cloud, lr=0.3, momentum=0.9, momentum_buf=buf,
                              momentum_init=True, grad_out=grad)
        agg.pop_step("p", step)
        np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(st.cloud))
        np.testing.assert_array_equal(bits(grad.cpu().numpy()), bits(st.grad))
        np.testing.assert_array_equal(bits(buf.cpu().numpy()), bits(st.buf))


def test_param_sharded_step_blocked(pg):
    """sharding.param_sharded_step on a column-blocked shard (the bench's
    layout and kernel) == the oracle, for a shard with a ragged tail."""
    from fedsim_amd import ops, sharding

    dev = torch.device("cuda", 0)
    K, Pfull, world = 300, 1_000_003, 3
    X = V.client_rows("realistic", K, Pfull, 8)
    w = V.client_weights("fedavg", K, 8)
    W = sum(w)
    avg_ref = ref.reduce(X, w, W=W)
    cloud0 = V.cloud_vector(Pfull, 9)
    exp = ref.fedavg_sgd(avg_ref, cloud0, 0.7)
    for r in range(world):
        lo, hi = sharding.shard_span(Pfull, r, world)
        Xs = torch.from_numpy(np.ascontiguousarray(X[:, lo:hi])).to(dev)
        C = ops.choose_block_cols(hi - lo)
        Xb = ops.to_blocked(Xs, C)
        cloud = torch.from_numpy(cloud0[lo:hi].copy()).to(dev)
        step = ops.ServerStep("fedavg", cloud, lr=0.7)
        sharding.param_sharded_step(Xb, sharding.weights_fp32(w, dev), W, step)
        np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(exp[lo:hi]))


@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("run", SYN_RUNS, ids=[f"{r['id']}-{r['algorithm']}" for r in SYN_RUNS])
def test_single_process_device_shards_round_loop(run, device, round_arrays):
    """ShardedSerialAggregator(devices=[...]): one process, three column
    shards (all on the box's one GPU here; on a node, one per GPU), with the
    cloud in HBM (steps in place) or on the host (each shard's step on a copy
    of its slice moved over the link, results assembled in pinned memory):
    the reference's 5-round trajectories, bitwise."""
    from functools import partial

    from fedsim_amd.sharding import ShardedSerialAggregator

    alg = _build(run, device, partial(ShardedSerialAggregator, devices=["cuda:0"] * 3,
                                      borrow=True, expected_rows=5))
    scores = alg.train(rounds=4)
    _check_run(run, alg.get_server_storage(), scores, round_arrays, device)


def test_single_process_device_shards_sources():
    """Host (pageable / pinned) vectors into one key and HBM vectors into
    another through three device shards: get mid-stream, pop to the host /
    the GPU, and pop_step with a momentum SGD step on a host-resident cloud,
    bitwise vs the oracle.  Host values into HIP shards are one device (the
    first value's); an HBM vector added to the host key raises, as the
    reference's host sum would, and the reverse."""
    from fedsim_amd import ops
    from fedsim_amd.sharding import ShardedSerialAggregator

    dev = torch.device("cuda", 0)
    K, P = 17, 300_007
    X = V.client_rows("realistic", K, P, 15)
    w = V.client_weights("fedavg", K, 15)
    hk = [k for k in range(K) if k % 3 != 2]
    dk = [k for k in range(K) if k % 3 == 2]
    wh, wd = [w[k] for k in hk], [w[k] for k in dk]
    avg_h, avg_d = ref.reduce(X[hk], wh, W=sum(wh)), ref.reduce(X[dk], wd, W=sum(wd))
    for final in ("pop", "step"):
        agg = ShardedSerialAggregator(devices=[dev] * 3, borrow=True)
        for k in range(K):
            src = torch.from_numpy(X[k].copy())
            if k % 3 == 1:
                src = src.pin_memory()
            elif k % 3 == 2:
                src = src.to(dev)
            agg.add("d" if k % 3 == 2 else "p", src, w[k])
            if k == 8:
                with pytest.raises(RuntimeError, match="same device"):
                    agg.add("p", torch.from_numpy(X[k].copy()).to(dev), w[k])
                with pytest.raises(RuntimeError, match="same device"):
                    agg.add("d", torch.from_numpy(X[k].copy()), w[k])
                sel = [i for i in hk if i <= k]
                ws = [w[i] for i in sel]
                mid = agg.get("p")
                np.testing.assert_array_equal(bits(mid.cpu().numpy()),
                                              bits(ref.reduce(X[sel], ws, W=sum(ws))))
        outd = agg.pop("d")
        assert outd.device == dev
        np.testing.assert_array_equal(bits(outd.cpu().numpy()), bits(avg_d))
        if final == "pop":
            out = agg.pop("p")
            assert out.device.type == "cpu"
            np.testing.assert_array_equal(bits(out.numpy()), bits(avg_h))
            continue
        cloud0 = V.cloud_vector(P, 16)
        st = ref.ServerState("fedavg", cloud0, dict(lr=0.3, momentum=0.9))
        st.step(avg_h)
        cloud = torch.from_numpy(cloud0.copy())
        grad, buf = torch.empty_like(cloud), torch.empty_like(cloud)
        agg.pop_step("p", ops.ServerStep("fedavg", cloud, lr=0.3, momentum=0.9,
                                         momentum_buf=buf, momentum_init=True, grad_out=grad))
        np.testing.assert_array_equal(bits(cloud.numpy()), bits(st.cloud))
        np.testing.assert_array_equal(bits(grad.numpy()), bits(st.grad))
        np.testing.assert_array_equal(bits(buf.numpy()), bits(st.buf))


# ---------------------------------------------------------------------------
# ClientShardedSerialAggregator (client-sharded rounds on the plugin surface)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["chain", "allreduce"])
@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("run", CS_RUNS, ids=[f"{r['id']}-{r['algorithm']}" for r in CS_RUNS])
def test_client_sharded_round_loop_one_rank_rccl(run, device, mode, pg, round_arrays):
    """The reference's 5-round trajectories through CentralFLAlgorithm with
    the client-sharded aggregator on a one-rank RCCL group: the message
    exchange, the HIP entry's partial sum, the collective (nothing to
    reorder at one rank: exact in both modes) and the server step."""
    from functools import partial

    from fedsim_amd.sharding import ClientShardedSerialAggregator

    alg = _build(run, device, partial(ClientShardedSerialAggregator, mode=mode, borrow=True,
                                      expected_rows=5))
    scores = alg.train(rounds=4)
    _check_run(run, alg.get_server_storage(), scores, round_arrays, f"{device} {mode}")


def _gloo_gpu_client_worker(rank, world, store, ids, mode, outdir):
    """One rank of a gloo group sharing cuda:0: trains its block of clients,
    HIP entries, the chain / all-reduce through host memory."""
    import json
    from functools import partial

    import torch.distributed as dist

    from fedsim_amd.sharding import ClientShardedSerialAggregator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        runs = {r["id"]: r for r in _golden_runs()}
        for rid in ids:
            alg = _build(runs[rid], "cuda", partial(ClientShardedSerialAggregator, mode=mode,
                                                    borrow=True))
            scores = alg.train(rounds=4)
            st = alg.get_server_storage()
            out = {}
            for name in ("cloud_params", "avg_params", "h"):
                t = st.read(name, silent=True)
                if isinstance(t, torch.Tensor):
                    out[name] = t.detach().cpu().numpy()
            np.savez(os.path.join(outdir, f"{rid}_rank{rank}.npz"), **out)
            with open(os.path.join(outdir, f"{rid}_rank{rank}.json"), "w") as f:
                json.dump({k: float(v) for k, v in scores.items()}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["chain", "allreduce"])
def test_client_sharded_round_loop_two_ranks_on_one_gpu(mode, round_arrays):
    """Two ranks (gloo, both on cuda:0) each train and reduce HALF of every
    round's clients with the HIP kernels: the chain gives the reference's
    5-round trajectories bit for bit on both ranks, the all-reduce within
    1e-6 normwise."""
    import json
    import tempfile

    import torch.multiprocessing as mp

    ids = [r["id"] for r in CS_RUNS]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_gpu_client_worker, args=(2, _file_store(d), ids, mode, d), nprocs=2,
                           join=True, start_method="spawn")
        for run in CS_RUNS:
            for r in range(2):
                got = np.load(os.path.join(d, f"{run['id']}_rank{r}.npz"))
                for name in got.files:
                    key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
                    if key not in round_arrays:
                        continue
                    want = round_arrays[key]
                    if mode == "chain":
                        np.testing.assert_array_equal(bits(got[name]), bits(want),
                                                      err_msg=f"{run['id']} rank {r} {name}")
                    else:
                        scale = np.linalg.norm(round_arrays[f"{run['id']}/cloud"]
                                               if name == "h" else want)
                        assert np.linalg.norm(got[name].astype(np.float64) - want) / scale <= 1e-6
                with open(os.path.join(d, f"{run['id']}_rank{r}.json")) as f:
                    scores = json.load(f)
                if mode == "chain":
                    assert scores == run["scores"]


def _gloo_gpu_feddf_worker(rank, world, store, mode, outdir):
    """One rank of a gloo group sharing cuda:0: a FedDF round loop on the
    reference's CNNs whose teachers are replayed per rank on the HIP kernels
    and combined by the client-sharded aggregator."""
    import json
    import random
    from functools import partial

    import torch.distributed as dist

    from conftest import GOLDEN_DIR
    from fedsim_amd import models
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.distributed.centralized.training import feddf
    from fedsim_amd.sharding import ClientShardedSerialAggregator
    from oracle import synthetic_fl as S

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        with open(os.path.join(GOLDEN_DIR, "feddf_cnn.json")) as f:
            G = json.load(f)
        for run in G["runs"]:
            record = []
            orig = feddf.ShardedTeachers.mean_logits

            def spy(self, x, _orig=orig):
                out = _orig(self, x)
                record.append(out.detach().cpu().numpy().copy())
                return out

            feddf.ShardedTeachers.mean_logits = spy
            try:
                cls = S.make_algorithm(training.FedDF)
                dm = S.ImageDataManager(G["num_clients"], run["image_shape"], run["num_classes"],
                                        G["valid_size"])
                random.seed(S.RANDOM_SEED)
                torch.manual_seed(S.TORCH_SEED)
                alg = cls(data_manager=dm, metric_logger=None, num_clients=G["num_clients"],
                          sample_scheme="uniform", sample_rate=G["sample_rate"],
                          model_def=partial(getattr(models, run["model"]),
                                            **run["model_kwargs"]),
                          epochs=1, criterion_def="CrossEntropyScore",
                          optimizer_def=partial(torch.optim.SGD, lr=G["lr"]), device="cuda",
                          global_epochs=G["global_epochs"],
                          aggregator_factory=partial(ClientShardedSerialAggregator, mode=mode,
                                                     borrow=True))
                alg.train(rounds=G["rounds"])
            finally:
                feddf.ShardedTeachers.mean_logits = orig
            st = alg.get_server_storage()
            np.savez(os.path.join(outdir, f"{run['id']}_rank{rank}.npz"),
                     targets=np.stack(record),
                     cloud=st.read("cloud_params").detach().cpu().numpy())
            with open(os.path.join(outdir, f"{run['id']}_rank{rank}.json"), "w") as f:
                json.dump(st.read("teacher_replay"), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["chain", "allreduce"])
def test_client_sharded_feddf_two_ranks_on_one_gpu(mode):
    """FedDF under client-sharded rounds with the HIP path: two ranks (gloo,
    both on cuda:0) each replay their own clients' teachers on the conv /
    pool / Linear kernels and reduce their logits with fedagg_reduce_f32
    onto the chain's running sum (or from +0 for the all-reduce).  Against
    the reference's own SimpleCNN2 / SimpleCNN FedDF rounds: targets within
    1e-5 (round 0) / 1e-4, cloud within 1e-4; both ranks hold the same
    bits; the replay was kept on both ranks."""
    import json
    import tempfile

    import torch.multiprocessing as mp

    from conftest import GOLDEN_DIR

    with open(os.path.join(GOLDEN_DIR, "feddf_cnn.json")) as f:
        G = json.load(f)
    with np.load(os.path.join(GOLDEN_DIR, "feddf_cnn.npz"), allow_pickle=False) as z:
        golden = {k: z[k] for k in z.files}
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_gpu_feddf_worker, args=(2, _file_store(d), mode, d), nprocs=2,
                           join=True, start_method="spawn")
        for run in G["runs"]:
            rid = run["id"]
            got = [dict(np.load(os.path.join(d, f"{rid}_rank{r}.npz"))) for r in range(2)]
            rep = [json.load(open(os.path.join(d, f"{rid}_rank{r}.json"))) for r in range(2)]
            np.testing.assert_array_equal(bits(got[1]["cloud"]), bits(got[0]["cloud"]))
            np.testing.assert_array_equal(bits(got[1]["targets"]), bits(got[0]["targets"]))
            want_t = golden[f"{rid}/targets"]
            rounds, nb = want_t.shape[:2]
            t = got[0]["targets"]
            per_round = t.shape[0] // rounds
            for rr in range(rounds):
                for b in range(nb):
                    w = want_t[rr, b]
                    err = (np.linalg.norm(t[rr * per_round + b].astype(np.float64) - w)
                           / np.linalg.norm(w))
                    print(f"{rid} {mode} round {rr} batch {b}: targets {err:.2e}")
                    assert err <= (1e-5 if rr == 0 else 1e-4), (rid, rr, b, err)
            cloud = got[0]["cloud"]
            e = (np.linalg.norm(cloud[::G["stride"]].astype(np.float64)
                                - golden[f"{rid}/cloud_sample"])
                 / np.linalg.norm(golden[f"{rid}/cloud_sample"]))
            assert e <= 1e-4, (rid, e)
            for r in rep:
                assert r["replayed"] and r["fallbacks"] == 0 and r["conv_launches"] > 0, r
            assert sum(r["teachers_local"] for r in rep) == 4


@pytest.mark.parametrize("where", ["host", "device"])
def test_chained_entry_grows_without_draining(where):
    """A client-sharded rank's snapshotted rows (borrow off, host or HBM
    sources) through several ring growths: the chain entry grows its ring by
    copying the pending rows instead of draining them from +0, so it can
    still continue another rank's running sum -- bitwise the oracle's
    arrival-order sum from that acc_in."""
    from fedsim_amd.sharding import ClientShardedSerialAggregator

    dev = torch.device("cuda:0")
    K, P = 37, 50_003
    X = V.client_rows("realistic", K, P, 31)
    w = V.client_weights("fedavg", K, 31)
    acc0 = V.cloud_vector(P, 32)
    agg = ClientShardedSerialAggregator(mode="chain")
    e = agg._local_entry("p", torch.empty(P, device=dev))
    assert e.keep_pending and e.Rmax > K
    for k in range(K):
        src = torch.from_numpy(X[k].copy())
        e.add(src if where == "host" else src.to(dev), w[k])
        src.fill_(float("nan"))  # snapshotted at add
    assert e.R >= K and e.acc is None and e.chainable()
    got = e.partial(torch.from_numpy(acc0.copy()).to(dev), W=sum(w))
    want = ref.reduce(X, w, acc_in=acc0.copy(), W=sum(w))
    np.testing.assert_array_equal(bits(got.cpu().numpy()), bits(want))


def _dtype_runs():
    import json

    from conftest import GOLDEN_DIR

    with open(os.path.join(GOLDEN_DIR, "generic_keys.json")) as f:
        return json.load(f)["dtype_runs"]


def _dtype_round(run, factory):
    import random
    from functools import partial

    from fedsim_amd.distributed.centralized import training
    from oracle import generic_cases as G
    from oracle import synthetic_fl as S

    cls = S.make_algorithm(getattr(training, run["algorithm"]))
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
              sample_scheme="uniform", sample_rate=S.SAMPLE_RATE,
              model_def=S.MODELS[run["model"]], epochs=1, criterion_def="CrossEntropyScore",
              optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device="cuda",
              aggregator_factory=factory, **run["alg_kwargs"])
    scores = alg.train(rounds=S.ROUNDS)
    st = alg.get_server_storage()
    cloud = st.read("cloud_params")
    got = dict(cloud=G.encode(cloud.detach()))
    if run["algorithm"] == "AdaBest":
        got["avg_params"] = G.encode(st.read("avg_params"))
    buf = st.read("optimizer").state[cloud].get("momentum_buffer")
    if buf is not None:
        got["momentum_buffer"] = G.encode(buf)
    return got, {k: G.encode(v) for k, v in scores.items()}


@pytest.mark.parametrize("dtype", ["bfloat16", "float16", "float64"])
def test_sharded_generic_key_one_rank(dtype, pg):
    """A bf16 / fp16 / fp64 key under the parameter-sharded aggregator (one
    RCCL rank): the slice reduced with the reference's arithmetic in HBM
    (_RefDeviceEntry), assembled by the all-gather; then an fp32 value makes
    the key leave it (collective get_sum, torch's promotion) -- bitwise the
    reference's CPU aggregation throughout."""
    from fedsim_amd.sharding import ShardedSerialAggregator, _ShardEntry
    from oracle.generic_cases import encode
    from oracle.reference_loop import ReferenceSerialAggregator

    dt = getattr(torch, dtype)
    dev = torch.device("cuda:0")
    K, P = 13, 70_001
    g = torch.Generator().manual_seed(9)
    X = [(torch.randn(P, generator=g, dtype=torch.float64) * 0.3).to(dt) for _ in range(K)]
    w = [int(v) for v in torch.randint(1, 300, (K,), generator=g)]
    agg, ref = ShardedSerialAggregator(borrow=True, max_rows=4), ReferenceSerialAggregator()
    for k in range(K):
        agg.add("p", X[k].to(dev), w[k])
        ref.add("p", X[k], w[k])
    e = agg._members["p"]
    assert isinstance(e, _ShardEntry) and e.ref
    assert encode(agg.get_sum("p")) == encode(ref.get_sum("p"))
    assert encode(agg.get("p")) == encode(ref.get("p"))
    f32 = torch.randn(P, generator=g)
    agg.add("p", f32.to(dev), 3)  # leaves the kernel: promotion as the reference
    ref.add("p", f32, 3)
    assert encode(agg.pop("p")) == encode(ref.pop("p"))


def _gloo_dtype_worker(rank, world, store, outdir):
    import json
    from functools import partial

    import torch.distributed as dist

    from fedsim_amd.sharding import ShardedSerialAggregator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        out = {}
        for run in _dtype_runs():
            got, scores = _dtype_round(run, partial(ShardedSerialAggregator, borrow=True))
            out[run["id"]] = dict(outputs=got, scores=scores)
        with open(os.path.join(outdir, f"dtype_rank{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


def test_sharded_dtype_rounds_two_ranks_on_one_gpu():
    """fp64 / bf16 models through the parameter-sharded round driver, two
    gloo ranks sharing the GPU: each rank reduces half of every fp64 / bf16
    client vector in HBM with the reference's arithmetic; after 5 rounds
    both hold the reference's server state bit for bit."""
    import json
    import tempfile

    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_dtype_worker, args=(2, _file_store(d), d), nprocs=2, join=True,
                           start_method="spawn")
        for r in range(2):
            with open(os.path.join(d, f"dtype_rank{r}.json")) as f:
                got = json.load(f)
            for run in _dtype_runs():
                assert got[run["id"]]["outputs"] == run["outputs"], (run["id"], r)
                assert got[run["id"]]["scores"] == run["scores"], (run["id"], r)


def test_client_storage_tensor_arrives_as_a_leaf():
    """A client-storage tensor another rank wrote (host copy, requires_grad)
    is moved to this rank's GPU as a LEAF that requires grad, as the
    reference's own storage would hold it (an optimizer accepts it and its
    .grad fills in)."""
    from fedsim_amd.distributed.centralized.centralized_fl_algorithm import _from_host

    host = torch.arange(4.0).requires_grad_(True)
    t = _from_host(("__fedsim_tensor__", host, "cuda", True), torch.device("cuda:0"))
    assert t.device.type == "cuda" and t.is_leaf and t.requires_grad
    opt = torch.optim.SGD([t], lr=0.5)
    (t * t).sum().backward()
    opt.step()
    assert torch.equal(t.detach().cpu(), torch.arange(4.0) - 0.5 * 2 * torch.arange(4.0))
