"""GPU probe: quick bitwise check of libfedagg against a torch-CPU restatement of
SerialAggregator.add/pop, then a tuning sweep of the exact-mode reduce kernel.

Run on the GPU box:  python tools/gpu_probe.py [--K 1000] [--P 25000000]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def cpu_restatement(X, w):
    acc = 0
    for k in range(X.shape[0]):
        acc = acc + X[k] * w[k]
    return acc


def parity(K, P, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(K, P, generator=g)
    w = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    ref_sum = cpu_restatement(X, w)
    ref_avg = ref_sum / sum(w)
    Xd = X.cuda()
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device="cuda")
    out = torch.empty(P, device="cuda")
    res = {}
    for name, fl in [("default", 0), ("u4", ops.tuning_flags(unroll=4)),
                     ("u16", ops.tuning_flags(unroll=16)), ("vpt2", ops.tuning_flags(vpt=2)),
                     ("nt", ops.tuning_flags(nt=True)), ("scalar", 0x8)]:
        ops.reduce_slab(Xd, w32, out, flags=fl)
        s = out.cpu()
        ops.reduce_slab(Xd, w32, out, W=sum(w), flags=fl)
        a = out.cpu()
        res[name] = bool(torch.equal(s.view(torch.int32), ref_sum.view(torch.int32))) and bool(
            torch.equal(a.view(torch.int32), ref_avg.view(torch.int32)))
    return res


def sweep(K, P, iters):
    ldx = (P + 63) // 64 * 64
    X = torch.empty(K, ldx, device="cuda")
    X.normal_(0, 1)
    w32 = torch.randint(50, 601, (K,), device="cuda").float()
    out = torch.empty(P, device="cuda")
    bytes_alg = 4.0 * K * P + 4.0 * P
    results = []
    for unroll in (4, 8, 16):
        for vpt in (1, 2):
            for nt in (False, True):
                fl = ops.tuning_flags(unroll=unroll, vpt=vpt, nt=nt)
                ops.reduce_slab(X[:, :P], w32, out, W=1.0, P=P, flags=fl)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    ops.reduce_slab(X, w32, out, W=1.0, P=P, flags=fl)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
                r = dict(unroll=unroll, vpt=vpt, nt=nt, ms=ms, GBps=bytes_alg / ms / 1e6)
                print(json.dumps(r), flush=True)
                results.append(r)
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    print("device:", torch.cuda.get_device_name(0), flush=True)
    for K, P in [(1, 1), (3, 5), (7, 1023), (64, 65537), (257, 4099), (5, 199210)]:
        print("parity", K, P, parity(K, P), flush=True)
    t = time.time()
    sweep(a.K, a.P, a.iters)
    print("sweep s", time.time() - t)


if __name__ == "__main__":
    main()
