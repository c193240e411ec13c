"""Tuning sweep of the exact-mode reduce kernel at the headline size, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24).

python tools/sweep_reduce.py [--K 1000] [--P 25000000] [--rounds 3]
"""
import argparse
import itertools
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--table", action="store_true", help="also time the row-table kernel")
    ap.add_argument("--only-default", action="store_true")
    ap.add_argument("--kcap-pad", type=int, default=0,
                    help="extra (unused) rows per column block of the blocked slab")
    ap.add_argument("--pad-pair", type=int, default=None,
                    help="also time a copy of the slab with this many extra rows, interleaved")
    ap.add_argument("--blocked", type=int, default=0,
                    help="time only the column-blocked layout with this C (1024/2048/4096)")
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    ldx = (P + 63) // 64 * 64
    X = torch.empty((K, ldx), device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    for k0 in range(0, K, 100):
        X[k0:k0 + 100].normal_(0, 1, generator=g)
    Xv = X[:, :P]
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    out = torch.empty(P, device=dev)
    ref = torch.empty(P, device=dev)
    ops.reduce_slab(Xv, w32, ref, W=1.0, flags=ops.tuning_flags(unroll=8, vpt=1))
    table = torch.tensor([Xv[k].data_ptr() for k in range(K)], dtype=torch.int64, device=dev)
    rows = [Xv[k] for k in range(K)]
    variants = [dict(unroll=u, vpt=v, nt=bool(n), table=False)
                for u, v, n in itertools.product((2, 4, 8), (1, 2, 4), (0, 1))]
    if a.table:
        variants += [dict(unroll=u, vpt=v, nt=True, table=True)
                     for u, v in ((4, 2), (8, 1), (2, 4), (4, 4))]
    Xb = None
    if a.blocked:
        C = a.blocked
        Xb = ops.to_blocked(Xv, C, kcap=K + a.kcap_pad)
        bss = {1024: (256,), 2048: (256, 512), 4096: (256, 512, 1024)}[C]
        variants = [dict(unroll=u, bs=b, nt=True, table=False, blocked=C, flat=f)
                    for u, b, f in itertools.product((2, 4, 8), bss, (False, True))]
        if C == 4096:  # ablation: weights staged in LDS instead of scalar loads
            variants.append(dict(unroll=4, bs=256, nt=True, table=False, blocked=C, flat=False,
                                 ldsw=True))
        if a.only_default:
            variants = [dict(unroll=4, bs=256, nt=True, table=False, blocked=C, flat=False)]
        del X, Xv, rows, table
        torch.cuda.empty_cache()
        slabs = {a.kcap_pad: Xb}
        if a.pad_pair is not None:
            # same data in a second slab with a different row capacity,
            # timed interleaved with the first (one process, rule 24)
            Xb2 = torch.zeros((Xb.shape[0], K + a.pad_pair, C), device=dev)
            Xb2[:, :K].copy_(Xb[:, :K])
            slabs[a.pad_pair] = Xb2
            variants = [dict(v, kcap_pad=p) for p in slabs for v in variants]
    alg = 4.0 * K * P + 4.0 * P
    times = {i: [] for i in range(len(variants))}
    for r in range(a.rounds):
        for i, var in enumerate(variants):
            fl = ops.tuning_flags(unroll=var["unroll"], vpt=var.get("vpt", 0), nt=var["nt"],
                                  bs=var.get("bs", 0), flat=var.get("flat", False),
                                  ldsw=var.get("ldsw", False))

            def run():
                if var.get("blocked"):
                    ops.reduce_blocked(slabs[var.get("kcap_pad", a.kcap_pad)], w32, out, B=K,
                                       W=1.0, flags=fl)
                elif var["table"]:
                    ops.reduce_rows(rows, w32, out, W=1.0, flags=fl, table=table)
                else:
                    ops.reduce_slab(Xv, w32, out, W=1.0, flags=fl)

            run()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
            if r == 0:
                assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), var
    res = []
    for i, var in enumerate(variants):
        ms = float(np.median(times[i]))
        res.append(dict(var, ms_median=ms, ms_min=float(np.min(times[i])),
                        GBps=alg / ms / 1e6))
    res.sort(key=lambda d: d["ms_median"])
    for d in res:
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
