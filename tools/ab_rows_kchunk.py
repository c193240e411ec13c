"""Borrowed-row reduction split into k-chunks chained through HBM.

Hypothesis under test: the ~12 % gap between borrowed rows
and the column-blocked slab at 1000 x 25 M comes from the number of distinct
rows (100 MB apart) in flight at once -- waves drift across all K rows, so
the chip touches K far-apart pages at a time (address translation / DRAM
page pressure), where the slab's drift stays inside one K*C*4-byte block.

Variant "kc<N>": rows 0..N-1 in one launch (FEDAGG_INIT), then N..2N-1 with
acc_in = out, ... (the chained batches of fedagg.h, in arrival order, so the
result is bit-identical), finalize on the last chunk.  Extra traffic: 8 P
bytes per additional chunk.  "slab" is the same rows packed into the
column-blocked slab (one launch), for a same-box comparison.

python tools/ab_rows_kchunk.py [--K 1000] [--P 25000000] [--chunks 1000,500,250]
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
    ap.add_argument("--chunks", default="1000,500,334,250,200,129,100,64,32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--no-slab", action="store_true")
    ap.add_argument("--nt", type=int, default=0, help="1: non-temporal row loads (the product default)")
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11)
    rows = [torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g) for _ in range(K)]
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    W = float(w32.sum().item())
    table = ops.row_table(rows, dev)
    out = torch.empty(P, device=dev)
    chunks = [int(c) for c in a.chunks.split(",") if int(c) > 0]
    nt = ops.FEDAGG_NT if a.nt else 0

    def run_chunked(kc):
        k0 = 0
        while k0 < K:
            n = min(kc, K - k0)
            last = k0 + n >= K
            ops.reduce_rows(rows[k0:k0 + n], w32[k0:k0 + n], out,
                            acc_in=None if k0 == 0 else out, W=W if last else None,
                            table=table[k0:k0 + n], checked=True, flags=nt)
            k0 += n

    variants = [(f"kc{kc}", (lambda kc=kc: run_chunked(kc))) for kc in chunks]
    Xb = None
    if not a.no_slab:
        C = ops.choose_block_cols(P)
        Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
        for k in range(K):
            ops.pack_row(rows[k], Xb, k)
        variants.append((f"slab_C{C}", lambda: ops.reduce_blocked(Xb, w32, out, W=W, flags=nt)))
    torch.cuda.synchronize()
    times = {n: [] for n, _ in variants}
    ref = None
    ok = {}
    for r in range(a.rounds):
        for name, fn in variants:
            if r == 0:
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                ok[name] = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.iters)
    alg = 4.0 * K * P + 4.0 * K + 4.0 * P  # rows + weights + out (one pass)
    for name, _ in variants:
        t = times[name]
        ms = float(np.median(t))
        print(json.dumps(dict(K=K, P=P, variant=name, ms_median=ms, ms_min=float(np.min(t)),
                              GBps=alg / ms / 1e6, bitwise_vs_first=ok[name])), flush=True)


if __name__ == "__main__":
    main()
