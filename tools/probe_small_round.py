"""Where the time of a small host-resident round goes (BASELINE config 1 as
the CLI runs it without a GPU-resident model: K=5 SimpleMLP vectors of
199 210 floats on the host, the cloud on the host): wall time per stage of
FedAvg.receive_from_client x K + FedAvg.optimize, by wrapping the
aggregator's stages with perf_counter (synchronising where the stage ends on
the GPU), median over --reps rounds; the reference's own arithmetic on the
same host for comparison.

python tools/probe_small_round.py [--K 5] [--P 199210] [--reps 30]
"""
import argparse
import collections
import functools
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_plugin_round import messages, reference_round  # noqa: E402

from fedsim_amd.distributed.centralized.training import FedAvg  # noqa: E402
from fedsim_amd.distributed.centralized.training import utils as tu  # noqa: E402
from fedsim_amd.utils import SerialAggregator, Storage  # noqa: E402
from fedsim_amd.utils import aggregators as A  # noqa: E402
from fedsim_amd.utils.handover import hand_over, handover_round  # noqa: E402

T = collections.defaultdict(list)


def wrap(obj, name, label):
    fn = getattr(obj, name)

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[label].append(time.perf_counter() - t0)
    setattr(obj, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=5)
    ap.add_argument("--P", type=int, default=199_210)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--borrow-host", type=int, default=1)
    ap.add_argument("--pinned-cloud", type=int, default=0,
                    help="a page-locked cloud, as the round driver's init_cloud makes it")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    wrap(A._Ingest, "_put_locked", "put")
    wrap(A._DeviceEntry, "_flush", "flush")
    wrap(A._DeviceEntry, "release", "release")
    wrap(tu, "_fused_server_step_host", "fused_server_step_host")
    cloud = torch.zeros(a.P)
    if a.pinned_cloud:
        cloud = cloud.pin_memory()
    cloud.requires_grad_()
    rounds = []
    for rep in range(a.reps + 3):
        msgs = messages(a.K, a.P, "cpu_run", dev, seed=11 + rep)
        st = Storage()
        st.write("cloud_params", cloud)
        st.write("optimizer", torch.optim.SGD(params=[cloud], lr=1.0))
        st.write("lr_scheduler", None)
        agg = SerialAggregator(expected_rows=a.K, borrow=True, borrow_host=bool(a.borrow_host))
        torch.cuda.synchronize()
        if rep == 3:
            T.clear()
        t0 = time.perf_counter()
        with handover_round():
            for k in range(a.K):
                msg, msgs[k] = msgs[k], None
                hand_over(msg["local_params"])
                FedAvg.receive_from_client(st, k, msg, "train", agg, None)
                del msg
        t1 = time.perf_counter()
        FedAvg.optimize(st, agg, None)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if rep >= 3:
            rounds.append((t1 - t0, t2 - t1, t2 - t0))
    med = lambda xs: statistics.median(xs) * 1e6  # noqa: E731
    out = dict(K=a.K, P=a.P, reps=a.reps, pinned_cloud=bool(a.pinned_cloud),
               receive_us=med([r[0] for r in rounds]), optimize_us=med([r[1] for r in rounds]),
               round_us=med([r[2] for r in rounds]),
               stages_us_per_call={k: med(v) for k, v in T.items()},
               stage_calls_per_round={k: len(v) / a.reps for k, v in T.items()})
    ref = reference_round(messages(a.K, a.P, "cpu_run", dev), a.P, reps=10)
    out["reference_round_us"] = ref * 1e6 if isinstance(ref, float) else ref
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
