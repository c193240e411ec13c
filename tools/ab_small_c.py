"""Column-block width below 1024 for the narrow kernels: with C = 128 and two
columns per lane, one one-wave workgroup owns a whole column block, so it
streams one contiguous K*512-byte region (the "small per-workgroup chunks"
regime of the read-stream probes).  Needs a build with
-DFEDAGG_ANY_C (valid_block_cols admits 128..16384).  Fused FedAvg round,
forced narrow mappings, one slab allocation reinterpreted per C, interleaved.
Timing only: the slab's logical contents differ per C.

python tools/ab_small_c.py tools/variants/libfedagg_anyc.so [--K 1000] [--P 25000000]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import _native, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--Cs", default="128,256,512,1024,4096")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.abspath(a.lib), mode=ctypes.RTLD_LOCAL)
    res, args = _native.SIGNATURES["fedagg_reduce_step_blocked_f32"]
    fn = lib.fedagg_reduce_step_blocked_f32
    fn.restype, fn.argtypes = res, args
    dev = torch.device("cuda:0")
    K, P = a.K, a.P
    Cs = [int(c) for c in a.Cs.split(",")]
    numel = max(-(-P // C) * K * C for C in Cs)
    buf = torch.empty(numel, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    for o in range(0, numel, 1 << 30):
        buf[o:o + (1 << 30)].normal_(0.0, 0.05, generator=g)
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    W32 = float(w32.sum().item())
    stream = torch.cuda.current_stream(dev).cuda_stream
    cloud = torch.zeros(P, device=dev)
    grad = torch.empty(P, device=dev)
    step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
    cases = []
    for C in Cs:
        for m, u in (("narrow2", 8), ("narrow2", 16), ("narrow1", 8)):
            if C < (128 if m == "narrow2" else 64):
                continue
            cases.append((C, m, u, ops.tuning_flags(unroll=u, nt=True, mapping=m)))
    times = [[] for _ in cases]
    for _ in range(a.rounds):
        for i, (C, m, u, fl) in enumerate(cases):
            def run():
                rc = fn(buf.data_ptr(), K, C, w32.data_ptr(), K, P, None, W32, 0x1 | 0x2 | fl,
                        ctypes.byref(step.args), stream)
                assert rc == 0, (rc, C, m, u)

            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
    alg = 4.0 * K * P + 4.0 * K + 12.0 * P
    for (C, m, u, _), t in zip(cases, times):
        ms = float(np.median(t))
        print(json.dumps(dict(K=K, P=P, C=C, mapping=m, unroll=u, ms_median=ms,
                              ms_min=float(np.min(t)), GBps=alg / ms / 1e6)), flush=True)


if __name__ == "__main__":
    main()
