"""Interleaved A/B of slab layouts for the exact reduce + FedAvg step at one
(K, P): column-blocked with C = 1024 / 2048 / 4096 (fused step kernel) and
row-major (plain reduce kernel, then the step epilogue is not fused there, so
only the reduce is compared across all four), each under the library's
default mapping and the wide one.  Same data in every layout; bitwise check.

python tools/ab_layout.py [--K 500] [--P 25000000] [--rounds 6]
(four copies of the K x P data are resident at once: 200 GB at the default)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=500)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    ldx = (P + 63) // 64 * 64
    X = torch.empty((K, ldx), device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    for k0 in range(0, K, 100):
        X[k0:k0 + 100].normal_(0, 0.05, generator=g)
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    W = float(w32.sum().item())
    out = torch.empty(P, device=dev)
    ref = torch.empty(P, device=dev)
    ops.reduce_slab(X[:, :P], w32, ref, W=W, P=P)
    variants = []
    for C in (4096, 2048, 1024):
        Xb = ops.to_blocked(X[:, :P], C)
        for m in ("auto", "wide"):
            fl = ops.tuning_flags(nt=True, mapping=m) | (ops.default_flags(C) if m == "wide" else 0)
            variants.append((f"blocked{C}/{m}", (lambda Xb=Xb, fl=fl:
                                                 ops.reduce_blocked(Xb, w32, out, W=W, flags=fl))))
    for m in ("auto", "wide"):
        fl = ops.tuning_flags(nt=True, mapping=m)
        variants.append((f"rowmajor/{m}", (lambda fl=fl: ops.reduce_slab(X[:, :P], w32, out, W=W,
                                                                         P=P, flags=fl))))
    for name, fn in variants:
        fn()
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), name
    times = {n: [] for n, _ in variants}
    for _ in range(a.rounds):
        for name, fn in variants:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 2)
    alg = 4.0 * K * P + 4.0 * K + 4.0 * P
    for name, _ in variants:
        ms = float(np.median(times[name]))
        print(json.dumps(dict(K=K, P=P, variant=name, ms_median=ms, GBps=alg / ms / 1e6)),
              flush=True)


if __name__ == "__main__":
    main()
