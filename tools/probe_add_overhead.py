"""Host cost per client of the plugin round's receive loop with HBM-resident
client vectors (tools/bench_plugin_round.py ``device_borrow``): the pieces
one ``FedAvg.receive_from_client`` runs, each timed over many calls with
perf_counter (median of 5 batches, microseconds per call).

python tools/probe_add_overhead.py [--K 1000] [--P 1085668]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_plugin_round import messages  # noqa: E402

from fedsim_amd.distributed.centralized.training import FedAvg  # noqa: E402
from fedsim_amd.utils import SerialAggregator, Storage  # noqa: E402
from fedsim_amd.utils.handover import hand_over, handover_round, take_token, unaliased  # noqa: E402


def per_call(fn, n, batches=5):
    out = []
    for _ in range(batches):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        out.append((time.perf_counter() - t0) / n * 1e6)
    return round(statistics.median(out), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=1_085_668)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t = torch.ones(a.P, device=dev)
    res = dict(K=a.K, P=a.P)
    res["current_device_us"] = per_call(torch.cuda.current_device, 20000)
    res["_cuda_getDevice_us"] = per_call(torch._C._cuda_getDevice, 20000)
    res["unaliased_us"] = per_call(lambda: unaliased(t), 20000)
    from fedsim_amd import ops

    h = torch.empty(2, a.P).pin_memory()
    res["host_mapped_us"] = per_call(lambda: ops.host_mapped(h), 5000)
    dd = torch.empty(2, a.P, device=dev)
    res["server_step_device_us"] = per_call(
        lambda: ops.ServerStep("fedavg", dd[0], lr=1.0, grad_out=dd[1]), 5000)
    res["server_step_mapped_us"] = per_call(
        lambda: ops.ServerStep("fedavg", h[0], lr=1.0, grad_out=h[1], device=dev), 5000)
    res["pinned_alloc_us"] = per_call(lambda: torch.empty(2, a.P, pin_memory=True), 2000)

    def tok():
        hand_over(t)
        take_token(t)
    with handover_round():
        res["hand_over_take_token_us"] = per_call(tok, 20000)

    def add_loop(borrow, declare, via_plugin):
        runs = []
        for _ in range(4):
            msgs = messages(a.K, a.P, "device_borrow", dev)
            st = Storage()
            agg = SerialAggregator(expected_rows=a.K, borrow=borrow)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with handover_round():
                for k in range(a.K):
                    msg, msgs[k] = msgs[k], None
                    if declare:
                        hand_over(msg["local_params"])
                    if via_plugin:
                        FedAvg.receive_from_client(st, k, msg, "train", agg, None)
                    else:
                        agg.add("local_params", msg["local_params"], msg["num_samples"]["train"])
                    del msg
            runs.append((time.perf_counter() - t0) / a.K * 1e6)
            del agg
            torch.cuda.synchronize()
        return round(statistics.median(runs[1:]), 2)

    res["add_borrow_us"] = add_loop(True, True, False)
    res["add_snap_us"] = add_loop(False, False, False)
    res["receive_borrow_declared_us"] = add_loop(True, True, True)
    res["receive_borrow_undeclared_us"] = add_loop(True, False, True)
    res["receive_snap_us"] = add_loop(False, False, True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
