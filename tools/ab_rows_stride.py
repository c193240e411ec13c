"""Borrowed-row rounds (fedagg_reduce_step_rows_f32) against the placement of
the client rows in HBM: K separate torch allocations (what a real round
borrows; the caching allocator rounds 100 MB up to 96 MiB = 3 * 2^25) versus
the same K rows laid out in one buffer at chosen strides (aligned like the
allocator, packed row-major, aligned + a per-row skew).  Fused FedAvg round,
auto mapping, interleaved; every variant checked bitwise against the first
on identical row contents (later rounds reuse the
shared buffer as the previous variant left it: timing only).

python tools/ab_rows_stride.py [--K 1000] [--P 25000000] [--rounds 5]
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
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--chunk-rows", type=int, default=10,
                    help="rows per allocation of the 'chunked' variant")
    ap.add_argument("--only", default="", help="comma-separated variant names")
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(9)
    sep = [torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g) for _ in range(K)]
    row_bytes = 4 * P
    aligned = -(-row_bytes // (2 << 20)) * (2 << 20)  # the allocator's 2 MiB rounding
    strides = {
        "buffer_aligned": aligned,
        "buffer_rowmajor": row_bytes,
        "buffer_aligned+256": aligned + 256,
        "buffer_aligned+4K": aligned + 4096,
        "buffer_aligned+16K": aligned + 16384,
        "buffer_aligned+64K+256": aligned + 65536 + 256,
    }
    chunk_name = f"chunked{a.chunk_rows}"
    want = set(a.only.split(",")) if a.only else set(strides) | {chunk_name}
    variants = [("separate", sep)]
    if chunk_name in want:  # rows carved from allocations of chunk_rows rows each
        chunks = []
        for k0 in range(0, K, a.chunk_rows):
            n = min(a.chunk_rows, K - k0)
            chunks.append(torch.empty(n * aligned // 4, device=dev))
        variants.append((chunk_name, [chunks[k // a.chunk_rows][(k % a.chunk_rows) * aligned // 4:][:P]
                                      for k in range(K)]))
    strides = {n: sb for n, sb in strides.items() if n in want}
    if strides:
        big = torch.empty(max(strides.values()) * K // 4 + P, device=dev)
        for name, sb in strides.items():
            variants.append((name, [big[k * sb // 4: k * sb // 4 + P] for k in range(K)]))
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    W = float(w32.sum().item())
    cloud0 = torch.empty(P, device=dev).normal_(0, 0.05, generator=g)
    cloud = torch.empty(P, device=dev)
    grad = torch.empty(P, device=dev)
    step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
    times = {n: [] for n, _ in variants}
    ref = None
    for r in range(a.rounds):
        for name, rows in variants:
            if name != "separate" and r == 0:  # same contents as the separate rows
                for k in range(K):
                    rows[k].copy_(sep[k])
            table = ops.row_table(rows, dev)
            cloud.copy_(cloud0)
            ops.reduce_rows_step(rows, w32, step, W=W, table=table, checked=True)
            torch.cuda.synchronize()
            if r == 0:
                if ref is None:
                    ref = cloud.clone()
                assert torch.equal(cloud.view(torch.int32), ref.view(torch.int32)), name
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops.reduce_rows_step(rows, w32, step, W=W, table=table, checked=True)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.iters)
    alg = 4.0 * K * P + 4.0 * K + 12.0 * P
    for name, _ in variants:
        t = times[name]
        ms = float(np.median(t))
        print(json.dumps(dict(K=K, P=P, variant=name, ms_median=ms, ms_min=float(np.min(t)),
                              GBps=alg / ms / 1e6)), flush=True)


if __name__ == "__main__":
    main()
