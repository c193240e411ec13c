"""Fused round (fedagg_reduce_step_blocked_f32: the step runs in the last
drain) against the split round (fedagg_reduce_blocked_f32 with the divide,
then fedagg_server_step_f32 on the stored average), both with the same
ServerStep operands and outputs, as SerialAggregator.pop_step issues them.
Interleaved per round, bitwise-checked against each other.

python tools/ab_fused_split.py [--K 1000[:K2...]] [--Ps 199210,1085668,...] [--algos fedavg,adabest]
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
    ap.add_argument("--K", default="1000", help="client counts, separated by : or ,")
    ap.add_argument("--Ps", default="199210,1085668,2097152,4194304,6250000,12500000,25000000")
    ap.add_argument("--algos", default="fedavg,adabest")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layout", default="blocked", choices=["blocked", "rows"],
                    help="rows: the borrowed path (fedagg_reduce_step_rows_f32 vs "
                         "fedagg_reduce_rows_f32 + fedagg_server_step_f32) over K separate tensors")
    a = ap.parse_args()
    for K in [int(x) for x in a.K.replace(":", ",").split(",")]:
        run(a, K)


def run(a, K):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    for P in [int(x) for x in a.Ps.replace(":", ",").split(",")]:
        C = ops.choose_block_cols(P)
        if a.layout == "rows":
            rows = [torch.empty(P, device=dev).normal_(0, 0.05, generator=g) for _ in range(K)]
            table = ops.row_table(rows, dev)
            Xb = rows
        else:
            Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev).normal_(0, 0.05, generator=g)
        w32 = torch.randint(50, 601, (K,), device=dev).float()
        W = float(w32.sum().item())
        iters = max(3, int(2e9 // (4 * K * P)))
        for algo in a.algos.split(","):
            cloud0 = torch.empty(P, device=dev).normal_(0, 0.05, generator=g)
            prev0 = torch.empty(P, device=dev).normal_(0, 0.05, generator=g)
            outs = {}
            for v in ("fused", "split"):
                cloud, prev = cloud0.clone(), prev0.clone()
                grad, avg = torch.empty(P, device=dev), torch.empty(P, device=dev)
                st = ops.ServerStep(algo, cloud, lr=1.0, coef=0.6 if algo == "adabest" else 0.0,
                                    aux=prev if algo == "adabest" else None, grad_out=grad)
                if a.layout == "rows" and v == "fused":
                    fn = (lambda st=st: ops.reduce_rows_step(rows, w32, st, W=W, table=table,
                                                             checked=True))
                elif a.layout == "rows":
                    fn = (lambda st=st, avg=avg: (ops.reduce_rows(rows, w32, avg, W=W, table=table,
                                                                  checked=True, flags=ops.FEDAGG_NT),
                                                  st.apply(avg)))
                elif v == "fused":
                    fn = (lambda st=st: ops.reduce_blocked_step(Xb, w32, st, W=W))
                else:
                    fn = (lambda st=st, avg=avg: (ops.reduce_blocked(Xb, w32, avg, W=W,
                                                                     flags=ops.FEDAGG_NT),
                                                  st.apply(avg)))
                fn()
                torch.cuda.synchronize()
                outs[v] = (fn, cloud, grad)
            same = all(torch.equal(outs["fused"][i].view(torch.int32), outs["split"][i].view(torch.int32))
                       for i in (1, 2))
            times = {v: [] for v in outs}
            for _ in range(a.rounds):
                for v, (fn, _, _) in outs.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[v].append(e0.elapsed_time(e1) / iters)
            alg = 4.0 * K * P
            r = dict(K=K, P=P, C=C, layout=a.layout, algo=algo, mapping=ops.column_mapping(P, B=K),
                     iters=iters,
                     first_round_bitwise_equal=same)
            for v in times:
                ms = float(np.median(times[v]))
                r[f"{v}_ms"] = ms
                r[f"{v}_GBps"] = alg / ms / 1e6
            r["split_over_fused"] = r["fused_ms"] / r["split_ms"]
            print(json.dumps(r), flush=True)
        del Xb
        rows = table = None
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
