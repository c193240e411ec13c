"""Host-resident FedSim rounds as the CLI runs them with ``--device cpu``:
real local SGD on every sampled client (the algorithm's own send_to_server,
local_updates.sgd_update: the reference's local_train loop,
fedsim/local/training/training.py:12-112), then the server aggregation --
timed two ways on the same host, same clients, same seeds:

  gpu   fedsim_amd's FedAvg round loop: each client's host vector is staged
        (pinned ring + copy stream) into the round's HBM slab at
        receive_from_client, reduced + stepped on the MI355X at optimize, the
        cloud kept on the host (config 1 as the CLI runs it);
  ref   the same round loop with the reference's server arithmetic on the
        host: the oracle's restatement of SerialAggregator (clone + mul + add
        per client, oracle/reference_loop.py; fedsim/utils/aggregators.py:
        23-40) and FedAvg.optimize's ``cloud.grad = cloud - avg;
        optimizer.step()`` (fedavg.py:193-208) on torch CPU.

Reported per leg and round: the round's wall time, the clients' training
time, the receive_from_client time (the GPU leg's staging memcpy + DMA issue;
the reference's clone + mul + add) and optimize.  The question this answers
(VERDICT r3 item 7): whether the per-client staging sits on the critical path
between one client's training and the next.

Synthetic data of the configs' shapes (no datasets offline): config 1 =
SimpleMLP on 1 x 28 x 28 (MNIST), 500 clients x 120 samples, K = 5; config 2
= SimpleCNN2(num_classes=100) on 3 x 24 x 24 (CIFAR-100 at the reference's
crop), 1000 clients x 50 samples, K = 10; fed-learn defaults otherwise
(epochs 5, batch 32, local SGD lr 0.1 wd 1e-3, server SGD lr 1.0;
fedsim_cli/fed_learn.py:58-161).

python tools/bench_host_rounds.py [--config 1|2] [--rounds 3] [--reps 2] [--legs gpu,ref]
"""
import argparse
import json
import os
import random
import sys
import time
from functools import partial

import torch
from torch.utils.data import TensorDataset

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = {
    1: dict(model="SimpleMLP", kw={}, shape=(1, 28, 28), classes=10, clients=500, samples=120),
    2: dict(model="SimpleCNN2", kw=dict(num_classes=100), shape=(3, 24, 24), classes=100,
            clients=1000, samples=50),
}


class SyntheticDM(object):
    """Per-client image tensors of the config's shape (seeded per client)."""

    def __init__(self, cfg):
        self.cfg = cfg

    def get_global_dataset(self):
        return {}

    def get_oracle_dataset(self):
        return {"train": list(range(self.cfg["clients"] * self.cfg["samples"]))}

    def get_local_splits_names(self):
        return ["train"]

    def get_local_dataset(self, cid):
        g = torch.Generator().manual_seed(1000 + cid)
        n = self.cfg["samples"]
        x = torch.randn((n,) + self.cfg["shape"], generator=g)
        y = torch.randint(0, self.cfg["classes"], (n,), generator=g)
        return {"train": TensorDataset(x, y)}


def timed(cls, clock):
    """The algorithm with its user methods timed (wall clock, synchronized
    where the GPU is involved)."""
    def wrap(name, fn):
        def f(*a, **k):
            t0 = time.perf_counter()
            out = fn(*a, **k)
            if name == "optimize" and torch.cuda.is_available():
                torch.cuda.synchronize()
            clock[name] = clock.get(name, 0.0) + time.perf_counter() - t0
            return out
        return staticmethod(f)

    return type("Timed" + cls.__name__, (cls,), {
        n: wrap(n, getattr(cls, n)) for n in ("send_to_server", "receive_from_client",
                                              "optimize")})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1, choices=[1, 2])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--legs", default="gpu,ref",
                    help="comma- or plus-separated: gpu (the round driver's aggregator: host vectors staged on the ingest "
                         "worker thread), gpu_sync (staged on the calling thread at add), ref")
    a = ap.parse_args()
    if a.threads:
        torch.set_num_threads(a.threads)
    from fedsim_amd import models
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.distributed.centralized.training import FedAvg
    from oracle.reference_loop import ReferenceSerialAggregator

    cfg = CONFIGS[a.config]
    torch.zeros(1, device="cuda")  # torch's HIP runtime first

    class RefFedAvg(FedAvg):
        """FedAvg.optimize as the reference writes it (fedavg.py:193-208)."""

        def optimize(server_storage, serial_aggregator, appendix_aggregator):
            if "local_params" in serial_aggregator:
                avg = serial_aggregator.pop("local_params")
                cloud = server_storage.read("cloud_params")
                opt = server_storage.read("optimizer")
                opt.zero_grad()
                cloud.grad = cloud.data - avg
                opt.step()
                sched = server_storage.read("lr_scheduler")
                if sched is not None:
                    sched.step()
            return serial_aggregator.pop_all()

    from fedsim_amd.utils import SerialAggregator

    K = int(0.01 * cfg["clients"])
    legs = {"gpu": (FedAvg, None), "ref": (RefFedAvg, ReferenceSerialAggregator),
            "gpu_sync": (FedAvg, partial(SerialAggregator, expected_rows=K, borrow=True,
                                         borrow_host=False))}
    out = []
    for rep in range(a.reps):
        for leg in a.legs.replace("+", ",").split(","):
            base, agg = legs[leg]
            clock = {}
            random.seed(7)
            torch.manual_seed(7)
            kw = {} if agg is None else dict(aggregator_factory=agg)
            alg = timed(base, clock)(
                data_manager=SyntheticDM(cfg), metric_logger=None, num_clients=cfg["clients"],
                sample_scheme="uniform", sample_rate=0.01,
                model_def=partial(getattr(models, cfg["model"]), **cfg["kw"]), epochs=5,
                criterion_def="CrossEntropyScore", batch_size=32,
                optimizer_def=partial(torch.optim.SGD, lr=1.0),
                local_optimizer_def=partial(torch.optim.SGD, lr=0.1, weight_decay=0.001),
                device="cpu", **kw)
            t0 = time.perf_counter()
            alg.train(rounds=a.rounds - 1)  # trange(rounds + 1): a.rounds rounds
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            cloud = alg.get_server_storage().read("cloud_params").detach()
            rec = dict(config=a.config, leg=leg, rep=rep, model=cfg["model"], K=K,
                       rounds=a.rounds, threads=torch.get_num_threads(),
                       round_ms=wall / a.rounds * 1e3,
                       train_ms_per_round=clock.get("send_to_server", 0) / a.rounds * 1e3,
                       receive_ms_per_round=clock.get("receive_from_client", 0) / a.rounds * 1e3,
                       receive_us_per_client=clock.get("receive_from_client", 0)
                       / (a.rounds * K) * 1e6,
                       optimize_ms_per_round=clock.get("optimize", 0) / a.rounds * 1e3,
                       cloud_norm=float(cloud.double().norm()))
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
