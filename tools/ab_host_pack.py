"""Interleaved A/B of how a page-locked host vector reaches its slab row
(aggregators._HOST_PACK): "dma" (a DMA into a device slot, then the HBM
pack; rounds 1-5) against "zero_copy" (the pack kernel reads the host vector
in place over PCIe, fedagg_pack_row_f32).  Same process, modes alternating
per repetition; wall time of whole plugin rounds (tools/bench_plugin_round.py)
and of host->host aggregation rounds at 25 M parameters (bench.py's
h2d_inclusive shape), every result checked bitwise between the modes.

python tools/ab_host_pack.py [--reps 5]
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
from bench_plugin_round import messages, one_round  # noqa: E402

from fedsim_amd.utils import SerialAggregator  # noqa: E402
from fedsim_amd.distributed.centralized.training import utils as U  # noqa: E402
from fedsim_amd.utils import aggregators as A  # noqa: E402

MODES = ("dma", "zero_copy")


def plugin_round(K, P, where, dev):
    cloud = torch.zeros(P, device="cpu" if where == "cpu_run" else dev, requires_grad=True)
    total = one_round(messages(K, P, where, dev), cloud, False)[1]
    return total, cloud.detach().cpu().clone()


def h2d_round(pool, K, w, pinned):
    agg = SerialAggregator(expected_rows=K, borrow_host=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        agg.add("p", pool[k % len(pool)], w[k])
    out = agg.pop("p")
    torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--h2d-only", action="store_true")
    ap.add_argument("--slots-ab", default="",
                    help="A/B the ingest ring's staging slots instead, e.g. 3:5 (host rounds)")
    ap.add_argument("--pack-modes", default="dma:zero_copy",
                    help="the two _HOST_PACK values compared (':'-separated)")
    ap.add_argument("--overlap-ab", action="store_true",
                    help="A/B aggregators._INGEST_OVERLAP instead (off = 'dma' column, "
                         "on = 'zero_copy' column), on the host-vector rounds")
    ap.add_argument("--step-ab", action="store_true",
                    help="A/B the host server step (training/utils._HOST_STEP) instead, "
                         "on the cloud-on-host rounds")
    ap.add_argument("--h2d-P", default="25000000", help="vector sizes, separated by :")
    a = ap.parse_args()
    global MODES
    dev = torch.device("cuda:0")
    rings = {}
    if a.slots_ab:
        MODES = tuple(a.slots_ab.split(":"))
        rings = {m: A._Ingest(dev, nslots=int(m)) for m in MODES}
    elif not (a.step_ab or a.overlap_ab):
        MODES = tuple(a.pack_modes.split(":"))
    res = {}
    cases = [("cfg1_cpu_run", 5, 199_210, "cpu_run", 30),
             ("cfg1_host_pageable", 5, 199_210, "host_pageable", 30),
             ("cfg2_K10_cpu_run", 10, 1_085_668, "cpu_run", 20),
             ("cfg2_K10_host_pinned", 10, 1_085_668, "host_pinned", 20),
             ("cfg2_K1000_host_pageable", 1000, 1_085_668, "host_pageable", 2)]
    if a.step_ab:
        cases = [c for c in cases if c[3] == "cpu_run"]
    if a.overlap_ab or a.slots_ab:
        cases = [("cfg2_K1000_host_pinned", 1000, 1_085_668, "host_pinned", 2),
                 ("cfg2_K1000_host_pageable", 1000, 1_085_668, "host_pageable", 2)]

    def set_mode(m):
        if rings:
            A._INGESTS[dev] = rings[m]
        elif a.step_ab:
            U._HOST_STEP = "zero_copy" if m == MODES[1] else "dma"
        elif a.overlap_ab:
            A._INGEST_OVERLAP = m == MODES[1]
        else:
            A._HOST_PACK = m
    for name, K, P, where, n in ([] if a.h2d_only else cases):
        times = {m: [] for m in MODES}
        outs = {}
        for rep in range(n + 1):
            for m in MODES:
                set_mode(m)
                t, c = plugin_round(K, P, where, dev)
                if rep:
                    times[m].append(t)
                outs[m] = c
        same = torch.equal(outs[MODES[0]].view(torch.int32), outs[MODES[1]].view(torch.int32))
        res[name] = {m: round(statistics.median(v) * 1e3, 3) for m, v in times.items()}
        res[name].update(unit="ms per round", bitwise_equal=same,
                         toggled="staging slots" if rings else "_HOST_STEP" if a.step_ab else
                         "_INGEST_OVERLAP" if a.overlap_ab else "_HOST_PACK")
        print(json.dumps({name: res[name]}), flush=True)
    for P, pinned in [(int(p), pin) for p in a.h2d_P.split(":") for pin in (True, False)
                      if not a.step_ab]:
        K = max(64, min(1000, int(64 * 25_000_000 // P)))  # >= 6.4 GB per round
        w = [50 + (37 * k) % 551 for k in range(K)]
        pool = [torch.empty(P).normal_() for _ in range(8)]
        if pinned:
            pool = [t.pin_memory() for t in pool]
        times = {m: [] for m in MODES}
        outs = {}
        for rep in range(a.reps + 1):
            for m in MODES:
                set_mode(m)
                t, out = h2d_round(pool, K, w, pinned)
                if rep:
                    times[m].append(t)
                outs[m] = out
        same = torch.equal(outs[MODES[0]].view(torch.int32), outs[MODES[1]].view(torch.int32))
        name = f"h2d_P{P}_K{K}_" + ("pinned" if pinned else "pageable")
        res[name] = {m: round(4.0 * K * P / statistics.median(v) / 1e9, 2) for m, v in times.items()}
        res[name].update(unit="GB/s", bitwise_equal=same,
                         toggled="staging slots" if rings else
                         "_INGEST_OVERLAP" if a.overlap_ab else "_HOST_PACK")
        print(json.dumps({name: res[name]}), flush=True)
        del pool, outs
    A._HOST_PACK, U._HOST_STEP, A._INGEST_OVERLAP = "auto", "zero_copy", True
    print(json.dumps({"all": res}), flush=True)


if __name__ == "__main__":
    main()
