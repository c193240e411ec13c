"""Interleaved A/B of the fused round (fedagg_reduce_step_blocked_f32, FedAvg
SGD) under forced column mappings at one (K, P): every round times each
variant back to back (3 launches by HIP events), so box drift hits all
variants alike.  Results bitwise-checked against the first variant.

python tools/ab_mapping.py [--K 1000] [--P 25000000] [--rounds 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

VARIANTS = [("auto", 0), ("wide", 0), ("narrow2", 8), ("narrow2", 16), ("narrow2", 32),
            ("narrow4", 8), ("narrow4", 16), ("narrow1", 8), ("narrow1", 16), ("narrow1", 32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    run(a.K, a.P, a.rounds)


def run(K, P, rounds):
    dev = torch.device("cuda:0")
    C = ops.choose_block_cols(P)
    Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    for b0 in range(0, Xb.shape[0], 256):
        Xb[b0:b0 + 256].normal_(0.0, 0.05, generator=g)
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    W = float(w32.sum().item())
    cloud0 = torch.empty(P, device=dev).normal_(0, 0.05, generator=g)
    steps, ref = [], None
    for mapping, u in VARIANTS:
        cloud = cloud0.clone()
        grad = torch.empty(P, device=dev)
        st = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
        ops.reduce_blocked_step(Xb, w32, st, W=W, mapping=mapping, unroll=u)
        torch.cuda.synchronize()
        if ref is None:
            ref = cloud.clone()
        assert torch.equal(cloud.view(torch.int32), ref.view(torch.int32)), mapping
        steps.append(st)
    times = [[] for _ in VARIANTS]
    for _ in range(rounds):
        for i, (mapping, u) in enumerate(VARIANTS):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                ops.reduce_blocked_step(Xb, w32, steps[i], W=W, mapping=mapping, unroll=u)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 3)
    alg = 4.0 * K * P + 4.0 * K + 12.0 * P
    for (mapping, u), t in zip(VARIANTS, times):
        ms = float(np.median(t))
        print(json.dumps(dict(K=K, P=P, C=C, mapping=mapping, unroll=u or "default",
                              ms_median=ms, ms_min=float(np.min(t)), GBps=alg / ms / 1e6)),
              flush=True)


if __name__ == "__main__":
    main()
