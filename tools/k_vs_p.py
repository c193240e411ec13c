"""Same bytes, different aspect: time the blocked reduce (EpiStore) at
K x P = const (default 25e9 fp32 = 100 GB) from short columns (K=250) to long
ones (K=10000), one kernel build, one slab allocation, C=4096, forced
narrow2 mappings, shapes interleaved per round.  Separates per-wave
start-up cost (waves live for K rows) from the streaming rate.

python tools/k_vs_p.py [--KP 25e9] [--rounds 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

KS = (250, 500, 1000, 2000, 5000, 10000)
MAPS = (("narrow2", 8), ("narrow2", 16))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--KP", type=float, default=25e9)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--C", type=int, default=4096)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = a.C
    shapes = [(K, int(a.KP) // K) for K in KS]
    numel = max(ops.blocked_shape(K, P, C)[0] * K * C for K, P in shapes)
    buf = torch.empty(numel, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    step = 1 << 30
    for o in range(0, numel, step):
        buf[o:o + step].normal_(0.0, 0.05, generator=g)
    maxK = max(KS)
    w32 = torch.randint(50, 601, (maxK,), device=dev).float()
    out = torch.empty(max(P for _, P in shapes), device=dev)
    cases = []
    for K, P in shapes:
        nb = ops.blocked_shape(K, P, C)[0]
        Xb = buf[:nb * K * C].view(nb, K, C)
        for m, u in MAPS:
            fl = ops.tuning_flags(unroll=u, nt=True, mapping=m)
            cases.append((K, P, m, u, Xb, fl))
    times = [[] for _ in cases]
    for _ in range(a.rounds):
        for i, (K, P, m, u, Xb, fl) in enumerate(cases):
            o = out[:P]
            ops.reduce_blocked(Xb, w32[:K], o, W=1.0, flags=fl)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                ops.reduce_blocked(Xb, w32[:K], o, W=1.0, flags=fl)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 3)
    for (K, P, m, u, _, _), t in zip(cases, times):
        ms = float(np.median(t))
        waves = -(-P // 128)
        print(json.dumps(dict(K=K, P=P, C=C, mapping=m, unroll=u, waves=waves,
                              ms_median=ms, ms_min=float(np.min(t)),
                              GBps=(4.0 * K * P + 4.0 * P) / ms / 1e6)), flush=True)


if __name__ == "__main__":
    main()
