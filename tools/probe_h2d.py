"""Probe of the host-side pieces of the H2D-inclusive round (bench.py
h2d_inclusive_leg): pageable vs pinned D2H of the average, single- vs
multi-threaded staging memmove, and the per-add wall time of the ingest
paths.  python tools/probe_h2d.py [--P 25000000]"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd.utils import SerialAggregator  # noqa: E402


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=25_000_000)
    a = ap.parse_args()
    P = a.P
    nb = 4.0 * P
    dev = torch.device("cuda:0")
    d = torch.randn(P, device=dev)
    res = {}
    res["d2h_pageable_GBps"] = nb / t(lambda: d.to("cpu")) / 1e9
    hp = torch.empty(P, pin_memory=True)
    res["d2h_pinned_GBps"] = nb / t(lambda: hp.copy_(d, non_blocking=True)) / 1e9
    src = torch.randn(P)
    dst = torch.empty(P, pin_memory=True)
    res["memmove_1t_GBps"] = nb / t(lambda: ctypes.memmove(dst.data_ptr(), src.data_ptr(), 4 * P)) / 1e9
    for nt in (2, 4, 8):
        pool = ThreadPoolExecutor(nt)
        step = (P + nt - 1) // nt

        def par():
            fs = [pool.submit(ctypes.memmove, dst.data_ptr() + 4 * i * step,
                              src.data_ptr() + 4 * i * step, 4 * max(0, min(step, P - i * step)))
                  for i in range(nt)]
            for f in fs:
                f.result()
        res[f"memmove_{nt}t_GBps"] = nb / t(par) / 1e9
        pool.shutdown()
    res["torch_copy_GBps"] = nb / t(lambda: dst.copy_(src)) / 1e9
    res["h2d_pinned_GBps"] = nb / t(lambda: d.copy_(dst, non_blocking=True)) / 1e9
    res["h2d_pageable_GBps"] = nb / t(lambda: d.copy_(src)) / 1e9
    # direct DMA from FRESH pageable tensors (no staging copy), vs staging
    fresh = [torch.randn(P) for _ in range(6)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x in fresh:
        d.copy_(x, non_blocking=True)
    torch.cuda.synchronize()
    res["h2d_pageable_fresh_GBps"] = len(fresh) * nb / (time.perf_counter() - t0) / 1e9
    del fresh
    # per-add wall time through the aggregator
    pool_p = [torch.randn(P) for _ in range(4)]
    pool_pin = [x.pin_memory() for x in pool_p]
    for name, pl, kw in (("pageable_borrow_host", pool_p, dict(borrow_host=True)),
                         ("pinned_borrow_host", pool_pin, dict(borrow_host=True)),
                         ("pageable_snapshot", pool_p, {}), ("pinned_snapshot", pool_pin, {})):
        for rep in range(3):
            agg = SerialAggregator(expected_rows=32, **kw)
            torch.cuda.synchronize()
            adds = []
            t0 = time.perf_counter()
            for k in range(32):
                s = time.perf_counter()
                agg.add("p", pl[k % 4], 1 + k)
                adds.append(time.perf_counter() - s)
            t1 = time.perf_counter()
            e = agg._members["p"]
            e._copies_issued()
            if e.copy_event is not None:
                e.copy_event.synchronize()
            t2 = time.perf_counter()
            out = agg.pop("p")
            t3 = time.perf_counter()
        res[name] = dict(add_ms_mean=sum(adds) / len(adds) * 1e3, add_ms_max=max(adds) * 1e3,
                         adds_ms=(t1 - t0) * 1e3, drain_ms=(t2 - t1) * 1e3, pop_ms=(t3 - t2) * 1e3,
                         GBps=32 * nb / (t3 - t0) / 1e9, out_pinned=out.is_pinned())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
