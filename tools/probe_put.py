"""Where one host-vector staging put of the ingest ring goes
(aggregators._Ingest._put_locked): the same steps timed one by one for K
cold pageable client vectors of P floats -- slot wait, staging copy (one
memmove / the multi-threaded split / torch's copy_), the H2D DMA issue, the
pack-kernel launch and the event -- and the per-vector wall time when the
whole put runs as the ingest worker runs it.

python tools/probe_put.py [--P 1085668] [--K 64]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

_POOL = ThreadPoolExecutor(3)


def _split_memmove(dst, src, nbytes, n):
    """memmove over n threads (ctypes releases the GIL): the round-6 variant
    measured against torch's copy_ here, then dropped."""
    step = (nbytes // n + 4095) & ~4095
    futs = [_POOL.submit(ctypes.memmove, dst + i * step, src + i * step,
                         min(step, nbytes - i * step)) for i in range(1, n) if i * step < nbytes]
    ctypes.memmove(dst, src, min(step, nbytes))
    for f in futs:
        f.result()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_085_668)
    ap.add_argument("--K", type=int, default=64)
    a = ap.parse_args()
    P, K = a.P, a.K
    dev = torch.device("cuda:0")
    C = ops.choose_block_cols(P)
    Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
    res = {"P": P, "K": K, "bytes": 4 * P}
    for mode in ("memmove1", "split4", "torch_copy"):
        srcs = [torch.randn(P) for _ in range(K)]  # cold: K x 4P bytes, written once
        big = torch.empty(64 << 20)  # evict the host caches between vectors
        hb = [torch.empty(P, pin_memory=True) for _ in range(3)]
        db = [torch.empty(P, device=dev) for _ in range(3)]
        ev = [None] * 3
        stream = torch.cuda.Stream(dev)
        t = {k: [] for k in ("wait", "copy", "dma", "pack", "event", "total")}
        torch.cuda.synchronize()
        for k in range(K):
            big.add_(1.0) if k % 8 == 0 else None
            i = k % 3
            t0 = time.perf_counter()
            if ev[i] is not None:
                ev[i].synchronize()
            t1 = time.perf_counter()
            if mode == "memmove1":
                ctypes.memmove(hb[i].data_ptr(), srcs[k].data_ptr(), 4 * P)
            elif mode == "split4":
                _split_memmove(hb[i].data_ptr(), srcs[k].data_ptr(), 4 * P, 4)
            else:
                hb[i].copy_(srcs[k])
            t2 = time.perf_counter()
            with torch.cuda.stream(stream):
                db[i].copy_(hb[i], non_blocking=True)
            t3 = time.perf_counter()
            ops.pack_row(db[i], Xb, k, stream=stream)
            t4 = time.perf_counter()
            e = torch.cuda.Event()
            e.record(stream)
            ev[i] = e
            t5 = time.perf_counter()
            for name, v in (("wait", t1 - t0), ("copy", t2 - t1), ("dma", t3 - t2),
                            ("pack", t4 - t3), ("event", t5 - t4), ("total", t5 - t0)):
                t[name].append(v)
        torch.cuda.synchronize()
        res[mode] = {name: round(statistics.median(v[4:]) * 1e6, 1) for name, v in t.items()}
        res[mode]["copy_GBps"] = round(4 * P / (res[mode]["copy"] * 1e-6) / 1e9, 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
