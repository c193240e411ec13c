"""Wide (f32x4 slots per lane) vs narrow (one / two columns per lane) column
mapping of the exact-mode reduce, over P and K, on the column-blocked slab
(the aggregator's layout, C from ops.choose_block_cols), plus the fused
FedAvg round (fedagg_reduce_step_blocked_f32) with the library's automatic
choice against each forced mapping.  Kernel time by HIP events, median of
--iters; every variant checked bit for bit against the wide one.

python tools/sweep_mapping.py [--P 199210,1085668,3125000,6250000] [--K 10,100,1000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

REDUCE = [("wide", 0), ("narrow1", 8), ("narrow1", 16), ("narrow1", 32), ("narrow2", 8),
          ("narrow2", 16), ("narrow2", 32)]
STEP = [("auto", 0), ("wide", 0), ("narrow1", 8), ("narrow1", 16), ("narrow2", 8),
        ("narrow2", 16), ("narrow2", 32)]


def kernel_ms(fn, iters):
    for _ in range(2):
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
    ap.add_argument("--P", default="199210,1085668,3125000,6250000")
    ap.add_argument("--K", default="10,100,1000")
    ap.add_argument("--iters", type=int, default=15)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for P in (int(v) for v in a.P.split(",")):
        for K in (int(v) for v in a.K.split(",")):
            C = ops.choose_block_cols(P)
            Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev).normal_(0, 0.05)
            w32 = torch.randint(50, 601, (K,), device=dev).float()
            W = float(w32.sum().item())
            out = torch.empty(P, device=dev)
            ref = torch.empty(P, device=dev)
            ops.reduce_blocked(Xb, w32, ref, W=W, flags=ops.tuning_flags(nt=True, mapping="wide"))
            res = []
            for mapping, u in REDUCE:
                fl = ops.tuning_flags(unroll=u, nt=True, mapping=mapping) | \
                    (ops.default_flags(C) if mapping == "wide" else 0)

                def run():
                    ops.reduce_blocked(Xb, w32, out, W=W, flags=fl)

                ms = kernel_ms(run, a.iters)
                assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), (P, K, mapping)
                alg = 4.0 * K * P + 4.0 * K + 4.0 * P
                res.append(dict(kind="reduce", mapping=mapping, unroll=u or "default", ms=ms,
                                GBps=alg / ms / 1e6))
            cloud0 = torch.empty(P, device=dev).normal_(0, 0.05)
            cloud_ref = None
            for mapping, u in STEP:
                cloud = cloud0.clone()
                grad = torch.empty(P, device=dev)
                step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
                ops.reduce_blocked_step(Xb, w32, step, W=W, mapping=mapping, unroll=u)
                torch.cuda.synchronize()
                if cloud_ref is None:
                    cloud_ref = cloud.clone()
                assert torch.equal(cloud.view(torch.int32), cloud_ref.view(torch.int32)), mapping
                ms = kernel_ms(lambda: ops.reduce_blocked_step(Xb, w32, step, W=W,
                                                               mapping=mapping, unroll=u),
                               a.iters)
                alg = 4.0 * K * P + 4.0 * K + 12.0 * P
                res.append(dict(kind="step", mapping=mapping, unroll=u or "default", ms=ms,
                                GBps=alg / ms / 1e6))
            for r in res:
                print(json.dumps(dict(P=P, K=K, C=C, **r)), flush=True)
            del Xb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
