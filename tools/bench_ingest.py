"""H2D-inclusive rate of one aggregation round through the drop-in
SerialAggregator: K client vectors arrive as HOST tensors (as from the
reference's CPU-side local trainers), are snapshotted / DMA'd into the
column-blocked HBM ring, reduced on the GPU, and the average comes back to the
host (D2H included) — ``add`` x K + ``pop``, end to end, wall clock.

Also times the HBM-resident variants (vectors already in HBM, e.g. GPU local
training): snapshotted into the slab by a D2D pack (device_d2d), or reduced in
place through the row-pointer kernel (device_borrow, SerialAggregator(borrow=
True)), and reports the PCIe H2D copy ceiling measured on the same box.

The HBM-resident legs use K DISTINCT device tensors (20 GB at the defaults),
far above the 256 MB MALL: a small pool re-read cyclically is served from
cache and reports rates above the HBM peak (round 1's 7.46 TB/s figure with
an 8-tensor pool was such a number).  The host legs cycle --pool host tensors:
their rate is PCIe-bound and host memory is read once per client either way.

python tools/bench_ingest.py [--K 200] [--P 25000000] [--pool 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd.utils import SerialAggregator  # noqa: E402


def h2d_ceiling(P, dev, n=8):
    src = torch.empty(P).pin_memory()
    dst = torch.empty(P, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return 4.0 * P * n / (time.perf_counter() - t0) / 1e9


def run_round(pool, weights, K, **agg_kw):
    agg = SerialAggregator(expected_rows=K, **agg_kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        agg.add("local_params", pool[k % len(pool)], weights[k])
    out = agg.pop("local_params")
    if out.device.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K, P = a.K, a.P
    weights = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    host = [torch.randn(P) for _ in range(a.pool)]
    res = dict(K=K, P=P, pool=a.pool, threads=torch.get_num_threads(),
               h2d_ceiling_GBps=h2d_ceiling(P, dev))
    g = torch.Generator(device=dev).manual_seed(5)

    def distinct_device_rows():
        return [torch.empty(P, device=dev).normal_(0.0, 1.0, generator=g) for _ in range(K)]

    res["device_rows"] = f"{K} distinct HBM tensors ({4.0 * K * P / 1e9:.0f} GB)"
    for name, make, kw in (("host_pageable", lambda: host, {}),
                           ("host_pinned", lambda: [t.pin_memory() for t in host], {}),
                           ("device_d2d", distinct_device_rows, {}),
                           ("device_borrow", distinct_device_rows, dict(borrow=True))):
        pool = make()
        run_round(pool, weights, min(K, 2 * a.pool), **kw)  # warm-up (allocations, pinned cache)
        ts = [run_round(pool, weights, K, **kw) for _ in range(a.reps)]
        t = min(ts)
        res[name] = dict(seconds=t, GBps=4.0 * K * P / t / 1e9)
        del pool
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
