"""Dtype-generic keys under the multi-GPU aggregators, rehearsed on CPU over
gloo (world sizes 2 and 3), against the REFERENCE's own transcripts and
rounds (tests/golden/generic_keys.json, tools/gen_golden_generic.py).

* ClientShardedSerialAggregator: every scenario of oracle/generic_cases.py
  with its N-d values split over the ranks in contiguous blocks (the other
  ranks' values as RemoteRow stand-ins).  fp32 keys run the exact chain (the
  C oracle as each rank's rows, tests/shard_oracle.py); every other key
  keeps the reference's arithmetic, its running sum passed from rank to rank
  as raw bytes.  Every rank's transcript must be the reference's, bit for
  bit, in both client_reduction modes (generic sums always chain).
* ShardedSerialAggregator: the same scenarios (every rank holds every
  value; generic keys are replicated, fp32 keys parameter-sharded).
* The round driver with an fp64 / bf16 model, clients split over the ranks:
  the reference's 5-round trajectories bit for bit on every rank.
"""
import json
import os
import tempfile

import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN_DIR

with open(os.path.join(GOLDEN_DIR, "generic_keys.json")) as _f:
    _GOLD = json.load(_f)


def _file_store(d):
    """A file rendezvous for the spawned gloo ranks: no TCP port to race for
    (a port picked free and then bound by the store can be taken in between)."""
    return "file://" + os.path.join(d, "pg_store")


def _scenario_worker(rank, world, store, kind, mode, outdir):
    import torch.distributed as dist

    from fedsim_amd.sharding import (ClientShardedSerialAggregator, RemoteRow,
                                     ShardedSerialAggregator)
    from oracle import generic_cases as G
    from shard_oracle import ChainOracleEntry, OracleEntry, oracle_step

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        out = {}
        for name, steps in G.scenarios().items():
            n = max(1, G.n_tensor_adds(steps))

            def wrap(j, t, n=n):
                owner = j * world // n  # contiguous blocks of the arrival order
                return t if owner == rank else RemoteRow(t.shape, t.dtype, "cpu", owner)

            if kind == "client":
                agg = ClientShardedSerialAggregator(mode=mode, entry_factory=ChainOracleEntry,
                                                    step_impl=oracle_step)
                out[name] = G.replay(agg, steps, wrap=wrap)
            else:
                agg = ShardedSerialAggregator(entry_factory=lambda part, a: OracleEntry(part, a))
                out[name] = G.replay(agg, steps)
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,mode", [("client", "chain"), ("client", "allreduce"),
                                       ("param", None)])
@pytest.mark.parametrize("world", [2, 3])
def test_generic_scenarios_every_rank(world, kind, mode):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_scenario_worker, args=(world, _file_store(d), kind, mode, d),
                           nprocs=world, join=True, start_method="spawn")
        for r in range(world):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                got = json.load(f)
            for name, want in _GOLD["transcripts"].items():
                assert got[name] == want, (kind, mode, world, r, name)


def _rounds_worker(rank, world, store, run_ids, mode, outdir):
    import random
    from functools import partial

    import torch
    import torch.distributed as dist

    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.sharding import ClientShardedSerialAggregator
    from oracle import generic_cases as G
    from oracle import synthetic_fl as S
    from shard_oracle import ChainOracleEntry

    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        runs = {r["id"]: r for r in _GOLD["dtype_runs"]}
        out = {}
        for rid in run_ids:
            run = runs[rid]
            cls = S.make_algorithm(getattr(training, run["algorithm"]))
            random.seed(S.RANDOM_SEED)
            torch.manual_seed(S.TORCH_SEED)
            alg = cls(data_manager=S.FakeDataManager(), metric_logger=None,
                      num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                      sample_rate=S.SAMPLE_RATE, model_def=S.MODELS[run["model"]], epochs=1,
                      criterion_def="CrossEntropyScore",
                      optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device="cpu",
                      # the fp32 hook only places the round on the host (no GPU
                      # here): these models' keys never reach it
                      aggregator_factory=partial(ClientShardedSerialAggregator, mode=mode,
                                                 entry_factory=ChainOracleEntry),
                      **run["alg_kwargs"])
            scores = alg.train(rounds=S.ROUNDS)
            st = alg.get_server_storage()
            cloud = st.read("cloud_params")
            got = dict(cloud=G.encode(cloud.detach()))
            buf = st.read("optimizer").state[cloud].get("momentum_buffer")
            if buf is not None:
                got["momentum_buffer"] = G.encode(buf)
            out[rid] = dict(outputs=got, scores={k: G.encode(v) for k, v in scores.items()})
        with open(os.path.join(outdir, f"rounds{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["chain", "allreduce"])
@pytest.mark.parametrize("world", [2, 3])
def test_generic_client_sharded_rounds(world, mode):
    """fp64 / bf16 models through the client-sharded round driver: each rank
    trains its block of every round's clients; the parameter keys keep the
    reference's arithmetic across the ranks.  Bitwise the reference's
    trajectory on every rank, in both modes.  (AdaBest is refused under
    client sharding)"""
    runs = [r for r in _GOLD["dtype_runs"] if r["algorithm"] != "AdaBest"]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rounds_worker,
                           args=(world, _file_store(d), [r["id"] for r in runs], mode, d),
                           nprocs=world, join=True, start_method="spawn")
        for r in range(world):
            with open(os.path.join(d, f"rounds{r}.json")) as f:
                got = json.load(f)
            for run in runs:
                g = got[run["id"]]
                want = {k: v for k, v in run["outputs"].items() if k != "avg_params"}
                assert g["outputs"] == want, (run["id"], r)
                assert g["scores"] == run["scores"], (run["id"], r)
