"""Multi-process (world_size 2 and 3) CPU rehearsal of the multi-GPU protocols
in fedsim_amd.sharding over the gloo backend.  The per-rank reduction is the
C oracle injected as ``local_reduce`` (no GPU here); what is tested is the
decomposition, the collectives and the ordering guarantees:
  param     concatenated shards == single-device reference, bitwise
  chain     client-sharded pipeline == single-device reference, bitwise
  allreduce client-sharded partial sums: normwise <= 1e-6 + forward-error bound
and, on the plugin surface, ShardedSerialAggregator (the per-rank state is the
C oracle, tests/shard_oracle.py): the reference's own 5-round trajectories of
FedAvg / AdaBest / FedNova / FedDyn through CentralFLAlgorithm, every rank
holding the full model after each round, bitwise against the goldens.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import bits
from oracle import ref
from oracle import vectors as V


def _file_store(d):
    """A file rendezvous for the spawned gloo ranks: no TCP port to race for
    (a port picked free and then bound by the store can be taken in between)."""
    return "file://" + os.path.join(d, "pg_store")


def oracle_reduce(X, w32, out, acc_in, W, flags):
    """CPU stand-in for the HIP kernel (same bits)."""
    Xn = np.ascontiguousarray(X.numpy())
    ai = None if acc_in is None else np.ascontiguousarray(acc_in.numpy()).copy()
    res = ref.reduce(Xn, [float(v) for v in w32.tolist()], acc_in=ai, W=W)
    out.copy_(torch.from_numpy(res))
    return out


def _worker(rank, world, store, K, P, mode, outdir):
    import torch.distributed as dist

    from fedsim_amd import sharding

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        X = torch.from_numpy(V.client_rows("normal", K, P, 21))
        w = V.client_weights("fedavg", K, 21)
        W = sum(w)
        if mode == "param":
            lo, hi = sharding.shard_range(P, rank, world, sharding.ALIGN)
            out = torch.empty(hi - lo)
            sharding.param_sharded(X[:, lo:hi], sharding.weights_fp32(w, "cpu"), W, out,
                                   local_reduce=oracle_reduce)
            # assemble on rank 0 for checking (not part of the data path)
            sizes = [sharding.shard_range(P, r, world, sharding.ALIGN) for r in range(world)]
            parts = [torch.empty(h - l_) for l_, h in sizes]
            if rank == 0:
                parts[0] = out
                for r in range(1, world):
                    dist.recv(parts[r], src=r)
            else:
                dist.send(out, dst=0)
            res = torch.cat(parts) if rank == 0 else None
        else:
            klo, khi = sharding.shard_range(K, rank, world)
            Xl = X[klo:khi].contiguous()
            wl = sharding.weights_fp32(w[klo:khi], "cpu")
            res = torch.empty(P)
            if mode == "chain":
                sharding.client_sharded_chain(Xl, wl, W, res, n_blocks=7,
                                              local_reduce=oracle_reduce)
            else:
                sharding.client_sharded_allreduce(Xl, wl, W, res, local_reduce=oracle_reduce)
        if res is not None:
            np.save(os.path.join(outdir, f"res{rank}.npy"), res.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["param", "chain", "allreduce"])
def test_sharded_protocols(mode, world):
    K, P = 23, 4099
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _file_store(d), K, P, mode, d), nprocs=world,
                           join=True, start_method="spawn")
        X = V.client_rows("normal", K, P, 21)
        w = V.client_weights("fedavg", K, 21)
        exp = ref.reduce(X, w, W=sum(w))
        got = np.load(os.path.join(d, "res0.npy"))
        if mode in ("param", "chain"):
            np.testing.assert_array_equal(bits(got), bits(exp))
            if mode == "chain":
                for r in range(1, world):
                    np.testing.assert_array_equal(
                        bits(np.load(os.path.join(d, f"res{r}.npy"))), bits(exp))
        else:
            x64 = X.astype(np.float64)
            w64 = np.array([np.float32(v) for v in w], dtype=np.float64)
            y64 = (w64[:, None] * x64).sum(0) / np.float64(np.float32(sum(w)))
            rel = np.linalg.norm(got - exp) / np.linalg.norm(exp)
            assert rel <= 1e-6
            gamma = K * 2.0 ** -24 / (1 - K * 2.0 ** -24)
            bound = (gamma * (np.abs(w64[:, None] * x64).sum(0)) / np.float32(sum(w))
                     + np.abs(y64) * 2.0 ** -23)
            assert np.all(np.abs(got.astype(np.float64) - y64) <= bound)


def test_shard_range_covers_and_aligns():
    from fedsim_amd.sharding import shard_range

    for n in (0, 1, 63, 64, 65, 1000, 25_000_000, 25_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world, 64) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
                assert b % 64 == 0 or b == n


# ---------------------------------------------------------------------------
# ShardedSerialAggregator through the round driver
# ---------------------------------------------------------------------------
def _rounds_worker(rank, world, store, run_ids, outdir):
    import json
    import random
    from functools import partial

    import torch.distributed as dist

    from conftest import GOLDEN_DIR
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.sharding import ShardedSerialAggregator
    from oracle import synthetic_fl as S
    import shard_oracle
    from shard_oracle import OracleEntry

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
            runs = {r["id"]: r for r in json.load(f)["runs"]}
        for rid in run_ids:
            run = runs[rid]
            cls = S.make_algorithm(getattr(training, run["algorithm"]))
            random.seed(S.RANDOM_SEED)
            torch.manual_seed(S.TORCH_SEED)
            alg = cls(data_manager=S.FakeDataManager(), metric_logger=None,
                      num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                      sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                      criterion_def="CrossEntropyScore",
                      optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]),
                      device="cpu",
                      aggregator_factory=partial(ShardedSerialAggregator,
                                                 entry_factory=OracleEntry),
                      **run["alg_kwargs"])
            scores = alg.train(rounds=S.ROUNDS)
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
            with open(os.path.join(outdir, f"{rid}_rank{rank}_calls.json"), "w") as f:
                json.dump(shard_oracle.CALLS, f)
            shard_oracle.CALLS.update(add=0, pop_step=0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_aggregator_round_loop_bitwise(world):
    import json

    from conftest import GOLDEN_DIR

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        runs = [r for r in json.load(f)["runs"]
                if r.get("client", "synthetic") == "synthetic" and r["algorithm"] != "FedDF"]
    ids = [r["id"] for r in runs]
    assert {r["algorithm"] for r in runs} >= {"FedAvg", "AdaBest", "FedNova", "FedDyn"}
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rounds_worker, args=(world, _file_store(d), ids, d), nprocs=world,
                           join=True, start_method="spawn")
        for run in runs:
            for r in range(world):
                got = np.load(os.path.join(d, f"{run['id']}_rank{r}.npz"))
                for name in ("cloud_params", "avg_params", "h"):
                    key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
                    if key not in arrays:
                        continue
                    np.testing.assert_array_equal(bits(got[name]), bits(arrays[key]),
                                                  err_msg=f"{run['id']} rank {r} {name}")
                with open(os.path.join(d, f"{run['id']}_rank{r}.json")) as f:
                    assert json.load(f) == run["scores"], run["id"]
                with open(os.path.join(d, f"{run['id']}_rank{r}_calls.json")) as f:
                    calls = json.load(f)
                # every rank reduced its own slice and ran the narrowed step
                # once per round (5 rounds)
                assert calls["pop_step"] == 5 and calls["add"] >= 5, (run["id"], calls)


def test_round_driver_shard_over_option():
    """shard_over selects the sharded per-round aggregator (opt-in); the
    default stays the one-GPU SerialAggregator even under a process group."""
    from functools import partial

    from fedsim_amd.distributed.centralized.training import FedAvg
    from fedsim_amd.sharding import ShardedSerialAggregator
    from fedsim_amd.utils import SerialAggregator
    from oracle import synthetic_fl as S

    def make(**kw):
        return FedAvg(data_manager=S.FakeDataManager(), metric_logger=None,
                      num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                      sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                      criterion_def="CrossEntropyScore", device="cpu", **kw)

    f = make()._aggregator_factory
    assert f.func is SerialAggregator and f.keywords == dict(expected_rows=5, borrow=True,
                                                             borrow_host=True)
    f = make(shard_over=["cuda:0", "cuda:1"])._aggregator_factory
    assert f.func is ShardedSerialAggregator and f.keywords["devices"] == ["cuda:0", "cuda:1"]
    f = make(shard_over="group")._aggregator_factory
    assert f.func is ShardedSerialAggregator and "group" not in f.keywords
    with pytest.raises(ValueError):
        make(shard_over="group", aggregator_factory=partial(SerialAggregator))
    from fedsim_amd.sharding import ClientShardedSerialAggregator

    f = make(shard_clients="group", client_reduction="allreduce")._aggregator_factory
    assert f.func is ClientShardedSerialAggregator and f.keywords["mode"] == "allreduce"
    assert "group" not in f.keywords and f.keywords["borrow"] and f.keywords["borrow_host"]
    with pytest.raises(ValueError):
        make(shard_clients="group", shard_over="group")
    with pytest.raises(ValueError):
        ClientShardedSerialAggregator(mode="tree")


def test_client_sharded_add_after_get_is_refused():
    """Solo (no process group): a get combines the key's rows; a later add
    would not reach that sum, so it raises instead of being dropped."""
    import numpy as np

    from fedsim_amd.sharding import ClientShardedSerialAggregator
    from shard_oracle import ChainOracleEntry, oracle_step

    from oracle import ref

    agg = ClientShardedSerialAggregator(entry_factory=ChainOracleEntry, step_impl=oracle_step)
    rows = [torch.randn(33) for _ in range(3)]
    for k, r in enumerate(rows[:2]):
        agg.add("local_params", r, 10 + k)
    got = agg.get("local_params")
    want = ref.reduce(np.stack([r.numpy() for r in rows[:2]]), [10, 11], W=21)
    np.testing.assert_array_equal(got.numpy().view(np.uint32), want.view(np.uint32))
    with pytest.raises(RuntimeError):
        agg.add("local_params", rows[2], 12)
    assert torch.equal(agg.pop("local_params"), got)


def _api_worker(rank, world, store, outdir):
    """Every SerialAggregator call on a parameter-sharded key, including
    shards that are empty (P < 64 * world), against the one-process oracle."""
    import json

    import torch.distributed as dist

    from fedsim_amd import ops
    from fedsim_amd.sharding import ShardedSerialAggregator
    from shard_oracle import OracleEntry

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    out = {}
    try:
        for P in (1, 63, 65, 130, 4099):
            K = 7
            X = V.client_rows("realistic", K, P, P)
            w = V.client_weights("fedavg", K, P)
            w[3] = 0  # a zero weight is added (its product is +0.0)
            agg = ShardedSerialAggregator(entry_factory=OracleEntry)
            for k in range(K):
                agg.add("p", torch.from_numpy(X[k].copy()), w[k])
                agg.add("clients.train.loss", 0.5 + k, w[k])  # host scalar key
                if k == 2:
                    out[f"{P}/get2"] = agg.get("p").numpy().tolist()
            out[f"{P}/sum"] = agg.get_sum("p").numpy().tolist()
            out[f"{P}/weight"] = agg.get_weight("p")
            out[f"{P}/keys"] = sorted(agg.keys())
            out[f"{P}/shard"] = agg.shard_of("p")
            cloud = torch.from_numpy(V.cloud_vector(P, 1))
            buf, grad = torch.empty(P), torch.empty(P)
            step = ops.ServerStep("fedavg", cloud, lr=0.3, momentum=0.9, momentum_buf=buf,
                                  momentum_init=True, grad_out=grad)
            agg.pop_step("p", step)
            out[f"{P}/cloud"] = cloud.numpy().tolist()
            out[f"{P}/buf"] = buf.numpy().tolist()
            rep = agg.pop_all()
            out[f"{P}/report"] = float(rep["clients.train.loss"])
            assert "p" not in agg
        with open(os.path.join(outdir, f"api{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


def test_sharded_aggregator_api_every_rank():
    import json

    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_api_worker, args=(world, _file_store(d), d), nprocs=world, join=True,
                           start_method="spawn")
        got = [json.load(open(os.path.join(d, f"api{r}.json"))) for r in range(world)]
    for P in (1, 63, 65, 130, 4099):
        K = 7
        X = V.client_rows("realistic", K, P, P)
        w = V.client_weights("fedavg", K, P)
        w[3] = 0
        exp2 = ref.reduce(X[:3], w[:3], W=sum(w[:3]))
        exps = ref.reduce(X, w)
        st = ref.ServerState("fedavg", V.cloud_vector(P, 1), dict(lr=0.3, momentum=0.9))
        st.step(ref.reduce(X, w, W=sum(w)))
        loss = sum((0.5 + k) * w[k] for k in range(K)) / sum(w)
        spans = []
        for r in range(world):
            g = got[r]
            np.testing.assert_array_equal(bits(np.array(g[f"{P}/get2"], np.float32)), bits(exp2))
            np.testing.assert_array_equal(bits(np.array(g[f"{P}/sum"], np.float32)), bits(exps))
            np.testing.assert_array_equal(bits(np.array(g[f"{P}/cloud"], np.float32)),
                                          bits(st.cloud))
            np.testing.assert_array_equal(bits(np.array(g[f"{P}/buf"], np.float32)), bits(st.buf))
            assert g[f"{P}/weight"] == sum(w)
            assert g[f"{P}/keys"] == ["clients.train.loss", "p"]
            assert g[f"{P}/report"] == loss
            spans.append(tuple(g[f"{P}/shard"]))
        # the shards tile [0, P): equal 64-aligned widths, empty past the end
        assert spans[0][0] == 0 and spans[-1][1] == P
        for (a, b), (c, e) in zip(spans, spans[1:]):
            assert b == c


# ---------------------------------------------------------------------------
# ClientShardedSerialAggregator through the round driver
# ---------------------------------------------------------------------------
def _client_rounds_worker(rank, world, store, run_ids, mode, outdir):
    import json
    import random
    from functools import partial

    import torch.distributed as dist

    from conftest import GOLDEN_DIR
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.sharding import ClientShardedSerialAggregator
    from oracle import synthetic_fl as S
    import shard_oracle
    from shard_oracle import ChainOracleEntry, oracle_step

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
            runs = {r["id"]: r for r in json.load(f)["runs"]}
        for rid in run_ids:
            run = runs[rid]
            trained = []
            base = getattr(training, run["algorithm"])
            synth = S.make_algorithm(base)

            def send_to_server(id, *a, _f=synth.send_to_server, **k):
                trained.append(id)
                return _f(id, *a, **k)

            cls = type("Counted" + base.__name__, (synth,),
                       {"send_to_server": staticmethod(send_to_server)})
            random.seed(S.RANDOM_SEED)
            torch.manual_seed(S.TORCH_SEED)
            alg = cls(data_manager=S.FakeDataManager(), metric_logger=None,
                      num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                      sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                      criterion_def="CrossEntropyScore",
                      optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]),
                      device="cpu",
                      aggregator_factory=partial(ClientShardedSerialAggregator, mode=mode,
                                                 entry_factory=ChainOracleEntry,
                                                 step_impl=oracle_step),
                      **run["alg_kwargs"])
            scores = alg.train(rounds=S.ROUNDS)
            st = alg.get_server_storage()
            out = {}
            for name in ("cloud_params", "avg_params", "h"):
                t = st.read(name, silent=True)
                if isinstance(t, torch.Tensor):
                    out[name] = t.detach().cpu().numpy()
            np.savez(os.path.join(outdir, f"{rid}_rank{rank}.npz"), **out)
            with open(os.path.join(outdir, f"{rid}_rank{rank}.json"), "w") as f:
                json.dump(dict(scores={k: float(v) for k, v in scores.items()},
                               trained=trained, calls=dict(shard_oracle.CALLS)), f)
            shard_oracle.CALLS.update(add=0, pop_step=0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["chain", "allreduce"])
@pytest.mark.parametrize("world", [2, 3])
def test_client_sharded_round_loop(world, mode):
    """Each rank trains only its block of every round's sampled clients (5 of
    20 per round here), receives every message (the others' vectors as
    stand-ins), and the blocks are combined: the reference's own 5-round
    FedAvg (lr 1.0 / 0.3), FedNova and FedDyn trajectories BITWISE
    with the chain, within 1e-6 normwise with the all-reduce; scores equal
    on every rank."""
    import json

    from conftest import GOLDEN_DIR

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        # AdaBest's clients read a running mean that every receive updates
        # (adabest.py:76-80,167-169): refused under client sharding (below)
        runs = [r for r in json.load(f)["runs"]
                if r.get("client", "synthetic") == "synthetic"
                and r["algorithm"] not in ("FedDF", "AdaBest")]
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_client_rounds_worker,
                           args=(world, _file_store(d), [r["id"] for r in runs], mode, d),
                           nprocs=world, join=True, start_method="spawn")
        for run in runs:
            trained = []
            for r in range(world):
                got = np.load(os.path.join(d, f"{run['id']}_rank{r}.npz"))
                with open(os.path.join(d, f"{run['id']}_rank{r}.json")) as f:
                    meta = json.load(f)
                trained.append(meta["trained"])
                for name in ("cloud_params", "avg_params", "h"):
                    key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
                    if key not in arrays:
                        continue
                    want = arrays[key]
                    if mode == "chain":
                        np.testing.assert_array_equal(bits(got[name]), bits(want),
                                                      err_msg=f"{run['id']} rank {r} {name}")
                    else:
                        scale = np.linalg.norm(arrays[f"{run['id']}/cloud"] if name == "h"
                                               else want)
                        err = np.linalg.norm(got[name].astype(np.float64) - want) / scale
                        assert err <= 1e-6, (run["id"], r, name, err)
                if mode == "chain":
                    assert meta["scores"] == run["scores"], run["id"]
                else:
                    for k, v in run["scores"].items():
                        assert meta["scores"][k] == pytest.approx(v, rel=1e-6), k
                assert meta["calls"]["pop_step"] == 5, meta["calls"]
            # the ranks trained disjoint blocks that cover every sampled client
            per_round = [len(t) for t in trained]
            assert sum(per_round) == 5 * 5 and all(n < 25 for n in per_round), per_round


def _client_extras_worker(rank, world, store, outdir):
    """Stateful clients, a diverged client and FedDF under client sharding."""
    import json
    import random
    from functools import partial

    import torch.distributed as dist

    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.sharding import ClientShardedSerialAggregator
    from oracle import synthetic_fl as S
    from shard_oracle import ChainOracleEntry, oracle_step

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    factory = partial(ClientShardedSerialAggregator, entry_factory=ChainOracleEntry,
                      step_impl=oracle_step)
    res = {}
    try:
        def make(cls, **kw):
            random.seed(S.RANDOM_SEED)
            torch.manual_seed(S.TORCH_SEED)
            return cls(data_manager=S.FakeDataManager(), metric_logger=None,
                       num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                       sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                       criterion_def="CrossEntropyScore", device="cpu",
                       aggregator_factory=factory, **kw)

        synth = S.make_algorithm(training.FedAvg)

        # (1) a client that keeps state in its own storage across rounds
        def stateful(id, rounds, storage, *a, _f=synth.send_to_server, **k):
            n = storage.read("count") or 0
            storage.write("count", n + 1)
            # an entry written on odd visits and removed on even ones
            # (Storage.remove must reach the other ranks too)
            if storage.read("flag") is not None:
                storage.remove("flag")
            else:
                storage.write("flag", torch.tensor([float(id)]))
            storage.write("seen_rounds", torch.cat([storage.read("seen_rounds"),
                                                    torch.tensor([float(rounds)])])
                          if n else torch.tensor([float(rounds)]))
            return _f(id, rounds, storage, *a, **k)

        alg = make(type("Stateful", (synth,), {"send_to_server": staticmethod(stateful)}))
        sampled = []
        orig = alg._sample_clients
        alg._sample_clients = lambda: sampled.append(orig()) or sampled[-1]
        alg.train(rounds=S.ROUNDS)
        res["count"] = {cid: alg._client_memory[cid].read("count") or 0
                        for cid in range(S.NUM_CLIENTS)}
        res["seen"] = {cid: (alg._client_memory[cid].read("seen_rounds").tolist()
                             if alg._client_memory[cid].read("seen_rounds") is not None else [])
                       for cid in range(S.NUM_CLIENTS)}
        res["sampled"] = sampled
        res["flag"] = {cid: alg._client_memory[cid].read("flag") is not None
                       for cid in range(S.NUM_CLIENTS)}

        # (2) a diverged client in the third round: every rank stops there
        def diverging(id, rounds, *a, _f=synth.send_to_server, **k):
            msg = _f(id, rounds, *a, **k)
            if rounds == 2 and id == sampled[2][3]:
                msg["diverged"] = True
            return msg

        alg = make(type("Diverging", (synth,), {"send_to_server": staticmethod(diverging)}))
        scores = alg.train(rounds=S.ROUNDS)
        res["diverged_rounds"] = alg.get_server_storage().read("rounds")
        res["diverged_cloud"] = alg.get_server_storage().read("cloud_params").detach().tolist()
        res["diverged_scores"] = {k: float(v) for k, v in scores.items()}

        # (4) real local SGD (the clients' own send_to_server): every rank
        # trains only its block and ends the round with the same model
        random.seed(S.RANDOM_SEED)
        torch.manual_seed(S.TORCH_SEED)  # the same initial model on every rank
        alg = training.FedAvg(data_manager=S.TensorDataManager(), metric_logger=None,
                              num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                              sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                              criterion_def="CrossEntropyScore", device="cpu",
                              aggregator_factory=factory)
        torch.manual_seed(S.TORCH_SEED + 100 + rank)  # each rank's own training RNG
        alg.train(rounds=1)
        res["local_sgd_cloud"] = alg.get_server_storage().read("cloud_params").detach().tolist()

        # (5) a client that raises on rank 1: every rank raises, none hangs
        def failing(id, rounds, *a, _f=synth.send_to_server, **k):
            if rank == 1 and rounds == 1:
                raise ValueError("client failure on rank 1")
            return _f(id, rounds, *a, **k)

        alg = make(type("Failing", (synth,), {"send_to_server": staticmethod(failing)}))
        try:
            alg.train(rounds=S.ROUNDS)
            res["failure"] = "none"
        except ValueError as e:
            res["failure"] = "own: " + str(e)
        except RuntimeError as e:
            res["failure"] = "other: " + str(e)

        # (3) AdaBest: a client's context (average_sample) depends on the
        # earlier clients' receive_from_client -> refused on every rank
        alg = make(S.make_algorithm(training.AdaBest))
        try:
            alg.train(rounds=0)
            res["adabest"] = "ran"
        except RuntimeError as e:
            res["adabest"] = str(e)
        # ... and runs when the check is off (the caller accepts round-start
        # contexts): every rank still ends with the same model
        alg = make(S.make_algorithm(training.AdaBest), check_client_context=False)
        alg.train(rounds=1)
        res["adabest_unchecked"] = alg.get_server_storage().read("cloud_params").detach().tolist()

        # (6) a client that consumes Python random on rank 1 only: the next
        # round's samples differ -> every rank raises, none hangs
        def drawing(id, rounds, *a, _f=synth.send_to_server, **k):
            if rank == 1:
                random.random()
            return _f(id, rounds, *a, **k)

        alg = make(type("Drawing", (synth,), {"send_to_server": staticmethod(drawing)}))
        try:
            alg.train(rounds=S.ROUNDS)
            res["desync"] = "ran"
        except RuntimeError as e:
            res["desync"] = str(e)[:60]

        # (7) rank 1 drained rows from +0 before the chain reached it: the
        # feasibility is agreed collectively, every rank raises, none hangs
        from shard_oracle import DrainedChainEntry

        def drained_factory(**kw):
            return ClientShardedSerialAggregator(
                entry_factory=DrainedChainEntry if rank == 1 else ChainOracleEntry,
                step_impl=oracle_step, **kw)

        random.seed(S.RANDOM_SEED)
        torch.manual_seed(S.TORCH_SEED)
        alg = synth(data_manager=S.FakeDataManager(), metric_logger=None,
                    num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                    sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                    criterion_def="CrossEntropyScore", device="cpu",
                    aggregator_factory=drained_factory)
        try:
            alg.train(rounds=0)
            res["drained"] = "ran"
        except RuntimeError as e:
            res["drained"] = str(e)[:60]

        # (7b) the same for the weight-1 row sums (FedDF's teacher targets)
        agg = ClientShardedSerialAggregator(
            entry_factory=DrainedChainEntry if rank == 1 else ChainOracleEntry,
            step_impl=oracle_step)
        try:
            agg.ordered_rows_sum(torch.ones(2, 5) * (rank + 1), [0, 1], 5)
            res["rows_drained"] = "ran"
        except RuntimeError as e:
            res["rows_drained"] = str(e)[:60]

        # (8) stateful clients and a divergence: clients after the diverged
        # one keep the storage they had before that round (the reference
        # never trained them)
        def stateful_diverging(id, rounds, storage, *a, _f=synth.send_to_server, **k):
            msg = stateful(id, rounds, storage, *a, _f=_f, **k)
            if rounds == 2 and id == sampled[2][1]:
                msg["diverged"] = True
            return msg

        alg = make(type("StatefulDiverging", (synth,),
                        {"send_to_server": staticmethod(stateful_diverging)}))
        alg.train(rounds=S.ROUNDS)
        res["div_count"] = {cid: alg._client_memory[cid].read("count") or 0
                            for cid in range(S.NUM_CLIENTS)}
        with open(os.path.join(outdir, f"extras_rank{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def test_client_sharded_state_divergence_and_refusal():
    """Client storages written on one rank reach every rank (the next round
    may train that client elsewhere); a diverged client stops the whole
    training on every rank at the same round with the same state, and the
    clients after it keep their pre-round storage; AdaBest, whose clients'
    context depends on the earlier clients of the round, is refused (and runs
    with the check off); ranks whose client samples drift apart, or a rank
    that cannot continue the chain, make every rank raise instead of hang;
    with real local SGD (each rank drawing its own random numbers) every rank
    still ends each round with the same model."""
    import json

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_client_extras_worker, args=(world, _file_store(d), d), nprocs=world,
                           join=True, start_method="spawn")
        res = [json.load(open(os.path.join(d, f"extras_rank{r}.json"))) for r in range(world)]
    assert res[1]["failure"] == "own: client failure on rank 1"
    assert res[0]["failure"].startswith("other:")
    for r in res[1:]:
        r.pop("failure")
    res[0].pop("failure")
    for r in res[1:]:
        assert r == res[0]
    sampled = res[0]["sampled"]
    for cid in range(20):
        times = [i for i, s in enumerate(sampled) if cid in s]
        assert res[0]["count"][str(cid)] == len(times)
        assert res[0]["seen"][str(cid)] == [float(i) for i in times]
        assert res[0]["flag"][str(cid)] == (len(times) % 2 == 1)
    assert res[0]["diverged_rounds"] == 2  # rounds 0 and 1 completed
    assert "depend on each other" in res[0]["adabest"], res[0]["adabest"]
    assert res[0]["desync"].startswith("the ranks of a client-sharded round sampled"), res[0]
    assert res[0]["drained"].startswith("client_reduction='chain': a rank drained"), res[0]
    assert res[0]["rows_drained"] == res[0]["drained"], res[0]
    # round 2 trained its clients up to the diverged one (position 1)
    want = {cid: len([i for i, s in enumerate(sampled) if cid in s and
                      (i < 2 or (i == 2 and s.index(cid) <= 1))]) for cid in range(20)}
    assert {int(k): v for k, v in res[0]["div_count"].items()} == want


# ---------------------------------------------------------------------------
# FedDF under client-sharded rounds: the reference's own CNN rounds
# ---------------------------------------------------------------------------
def _feddf_worker(rank, world, store, mode, outdir):
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
    from shard_oracle import ChainOracleEntry, oracle_step

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
                          optimizer_def=partial(torch.optim.SGD, lr=G["lr"]), device="cpu",
                          global_epochs=G["global_epochs"],
                          aggregator_factory=partial(ClientShardedSerialAggregator, mode=mode,
                                                     entry_factory=ChainOracleEntry,
                                                     step_impl=oracle_step))
                scores = alg.train(rounds=G["rounds"])
            finally:
                feddf.ShardedTeachers.mean_logits = orig
            st = alg.get_server_storage()
            np.savez(os.path.join(outdir, f"{run['id']}_rank{rank}.npz"),
                     targets=np.stack(record),
                     cloud=st.read("cloud_params").detach().numpy(),
                     model=torch.nn.utils.parameters_to_vector(
                         st.read("model").parameters()).detach().numpy())
            with open(os.path.join(outdir, f"{run['id']}_rank{rank}.json"), "w") as f:
                json.dump(dict(scores={k: float(v) for k, v in scores.items()},
                               replay=st.read("teacher_replay")), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(3, "chain"), (2, "allreduce")])
def test_client_sharded_feddf_matches_reference(world, mode):
    """FedDF with each rank training and replaying only its own clients'
    teachers (K=4 per round over 2 / 3 ranks), the per-rank logit sums
    combined by the round's aggregator (feddf.py:117-142): against the
    reference's own SimpleCNN2(num_classes=100) / SimpleCNN FedDF rounds
    (tests/golden/feddf_cnn.*).  chain: targets within 1e-5 (round 0) /
    1e-4, cloud within 1e-4 normwise -- bitwise (cloud SHA-256, targets, scores)
    on the host that made the goldens; allreduce (reordered sum): the same
    normwise bounds.  Every rank ends with the same cloud and the same model
    (the last teacher, broadcast from its rank)."""
    import json

    from conftest import GOLDEN_DIR
    from oracle import synthetic_fl as S

    with open(os.path.join(GOLDEN_DIR, "feddf_cnn.json")) as f:
        G = json.load(f)
    same_host = G.get("host") == S.host_signature()
    with np.load(os.path.join(GOLDEN_DIR, "feddf_cnn.npz"), allow_pickle=False) as z:
        golden = {k: z[k] for k in z.files}
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_feddf_worker, args=(world, _file_store(d), mode, d), nprocs=world,
                           join=True, start_method="spawn")
        for run in G["runs"]:
            rid = run["id"]
            got = [dict(np.load(os.path.join(d, f"{rid}_rank{r}.npz"))) for r in range(world)]
            meta = [json.load(open(os.path.join(d, f"{rid}_rank{r}.json")))
                    for r in range(world)]
            for r in range(1, world):
                np.testing.assert_array_equal(bits(got[r]["cloud"]), bits(got[0]["cloud"]))
                np.testing.assert_array_equal(bits(got[r]["model"]), bits(got[0]["model"]))
                np.testing.assert_array_equal(bits(got[r]["targets"]), bits(got[0]["targets"]))
                assert meta[r]["scores"] == meta[0]["scores"]
            want_t = golden[f"{rid}/targets"]  # [rounds, batches, B, classes]
            rounds, nb = want_t.shape[:2]
            t = got[0]["targets"]
            per_round = t.shape[0] // rounds
            assert per_round in (nb, nb * G["global_epochs"]), t.shape
            for rr in range(rounds):
                for b in range(nb):
                    g, w = t[rr * per_round + b].astype(np.float64), want_t[rr, b]
                    err = np.linalg.norm(g - w) / np.linalg.norm(w)
                    assert err <= (1e-5 if rr == 0 else 1e-4), (rid, rr, b, err)
                    if mode == "chain" and same_host:
                        np.testing.assert_array_equal(bits(t[rr * per_round + b]), bits(w))
            cloud = got[0]["cloud"]
            e = (np.linalg.norm(cloud[::G["stride"]].astype(np.float64)
                                - golden[f"{rid}/cloud_sample"])
                 / np.linalg.norm(golden[f"{rid}/cloud_sample"]))
            assert e <= 1e-4, (rid, e)
            if mode == "chain" and same_host:
                assert V.sha256(cloud) == run["cloud_sha256"], rid
                assert meta[0]["scores"] == run["scores"]
            rep = meta[0]["replay"]
            assert rep["teachers_total"] == 4 and rep["client_reduction"] == mode
            assert sum(m["replay"]["teachers_local"] for m in meta) == 4
