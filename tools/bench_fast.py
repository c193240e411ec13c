"""Exact (default) vs FEDAGG_FAST (split-K, reordered) kernel time of the
plain blocked reduce at small P, where one column per lane cannot fill the
chip.  Kernel time by HIP events, median of --iters.

python tools/bench_fast.py [--P 1000,7850,50000,199210] [--K 100,1000,10000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def kernel_ms(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", default="1000,7850,50000,199210")
    ap.add_argument("--K", default="100,1000,10000")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for P in (int(v) for v in a.P.split(",")):
        for K in (int(v) for v in a.K.split(",")):
            C = ops.choose_block_cols(P)
            Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev).normal_(0, 0.05)
            w32 = torch.randint(50, 601, (K,), device=dev).float()
            W = float(w32.sum().item())
            out = torch.empty(P, device=dev)
            res = {}
            for name, fl in (("exact", ops.default_flags(C)),
                             ("fast", ops.default_flags(C) | ops.FEDAGG_FAST)):
                ms = kernel_ms(lambda: ops.reduce_blocked(Xb, w32, out, W=W, flags=fl), a.iters)
                res[name] = dict(ms=ms, GBps=(4.0 * K * P + 4.0 * K + 4.0 * P) / ms / 1e6)
            print(json.dumps(dict(K=K, P=P, **res)), flush=True)
            del Xb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
