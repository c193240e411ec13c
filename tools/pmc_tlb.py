"""Translation (UTCL1) behaviour of the three client-row layouts the reduce
kernels read, same data, same K x P, interleaved in one process: the
column-blocked slab (fedagg_reduce_blocked_f32), one row-major [K, P]
allocation (fedagg_reduce_f32) and K separate allocations through a row
pointer table (fedagg_reduce_rows_f32: borrowed client tensors).  Prints the
HIP-event time per launch; run under ``rocprofv3 --pmc
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY`` for the counters per kernel.

python tools/pmc_tlb.py [--K 600] [--P 25000000] [--iters 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=600)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    C = ops.choose_block_cols(P)
    Xb = torch.zeros(ops.blocked_shape(K, P, C), device=dev)
    X = torch.empty((K, P), device=dev)
    rows = []
    for k in range(K):  # K separate allocations, like borrowed client tensors
        r = torch.empty(P, device=dev).normal_(0, 1, generator=g)
        rows.append(r)
        X[k].copy_(r)
        ops.pack_row(r, Xb, k)
    table = ops.row_table(rows, dev)
    w32 = torch.randint(50, 601, (K,), device=dev, generator=g).float()
    W = float(w32.sum().item())
    nt = ops.FEDAGG_NT
    wide = ops.tuning_flags(mapping="wide", nt=True)
    names = ("blocked", "rowmajor", "rows", "rowmajor_nt", "rows_nt", "rows_wide_nt")
    outs = {n: torch.empty(P, device=dev) for n in names}
    run = {
        "blocked": lambda: ops.reduce_blocked(Xb, w32, outs["blocked"], W=W,
                                              flags=ops.default_flags(C)),
        "rowmajor": lambda: ops.reduce_slab(X, w32, outs["rowmajor"], W=W),
        "rows": lambda: ops.reduce_rows(rows, w32, outs["rows"], W=W, table=table, checked=True),
        "rowmajor_nt": lambda: ops.reduce_slab(X, w32, outs["rowmajor_nt"], W=W, flags=nt),
        "rows_nt": lambda: ops.reduce_rows(rows, w32, outs["rows_nt"], W=W, table=table,
                                           checked=True, flags=nt),
        "rows_wide_nt": lambda: ops.reduce_rows(rows, w32, outs["rows_wide_nt"], W=W,
                                                table=table, checked=True, flags=wide),
    }
    times = {n: [] for n in run}
    for _ in range(a.iters):
        for n, fn in run.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1))
    same = all(torch.equal(outs["blocked"], o) for o in outs.values())
    for n, ts in times.items():
        ms = min(ts)
        print(json.dumps(dict(layout=n, K=K, P=P, ms=ms, all_ms=ts,
                              gbps=4.0 * K * P / ms / 1e6, bitwise_equal=same)), flush=True)


if __name__ == "__main__":
    main()
