"""Kernel time of the fused round (fedagg_reduce_step_blocked_f32, FedAvg SGD
epilogue) at the reference's model sizes over a range of K: where the
column-parallel exact reduction under-fills the chip (P/4 float4 slots is the
only parallelism an in-order per-column sum has).

python tools/bench_smallp.py [--P 199210,1085668] [--K 10,50,100,500,1000]
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
    ap.add_argument("--P", default="199210,1085668")
    ap.add_argument("--K", default="10,50,100,500,1000")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--C", type=int, default=0, help="column block (default: ops.choose_block_cols)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for P in (int(v) for v in a.P.split(",")):
        for K in (int(v) for v in a.K.split(",")):
            C = a.C or ops.choose_block_cols(P)
            Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev).normal_(0, 0.05)
            w32 = torch.randint(50, 601, (K,), device=dev).float()
            W = float(w32.sum().item())
            cloud = torch.zeros(P, device=dev)
            grad = torch.empty(P, device=dev)
            step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
            for _ in range(3):
                ops.reduce_blocked_step(Xb, w32, step, W=W)
            torch.cuda.synchronize()
            ms = []
            for _ in range(a.iters):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.reduce_blocked_step(Xb, w32, step, W=W)
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            med = float(np.median(ms))
            alg = 4.0 * K * P + 4.0 * K + 12.0 * P
            print(json.dumps(dict(K=K, P=P, C=C, workgroups=(P + C - 1) // C, ms_median=med,
                                  ms_min=float(np.min(ms)), GBps=alg / med / 1e6)), flush=True)
            del Xb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
