"""cProfile of one end-to-end plugin round (tools/bench_plugin_round.py):
where the host time of receive_from_client x K + optimize goes.

python tools/profile_plugin_round.py [--K 1000] [--P 1085668] [--borrow 1]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_plugin_round import headline_round, messages, one_round  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=1_085_668)
    ap.add_argument("--borrow", type=int, default=1)
    ap.add_argument("--where", default=None,
                    help="device_borrow | device_snap | host_pinned | host_pageable | cpu_run "
                         "| gpu_clients")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    where = a.where or ("device_borrow" if a.borrow else "device_snap")
    pr = cProfile.Profile()
    if where == "gpu_clients":  # vectorize into slab rows (bench_plugin_round.headline_round)
        headline_round(a.K, a.P, dev, "slab_rows", 1)
        pr.enable()
        headline_round(a.K, a.P, dev, "slab_rows", 2)
        pr.disable()
    else:
        cloud = torch.zeros(a.P, device="cpu" if where == "cpu_run" else dev,
                            requires_grad=True)
        for _ in range(2):  # one_round consumes its messages
            one_round(messages(a.K, a.P, where, dev), cloud, bool(a.borrow))
        batches = [messages(a.K, a.P, where, dev) for _ in range(3)]
        pr.enable()
        for msgs in batches:
            one_round(msgs, cloud, bool(a.borrow))
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
