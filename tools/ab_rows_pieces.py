"""Probe A/B for the borrowed-rows gap (tools/rows_pieces.hip): one wave reads
N consecutive 512-byte pieces of each row per visit (N * 512 contiguous bytes)
over K separate row allocations and over the column-blocked slab holding the
same rows; the product kernels (fedagg_reduce_rows_f32 / _blocked_f32, nt)
alongside.  Probe outputs are checked bitwise against each other.

python tools/ab_rows_pieces.py [--K 1000] [--P 25000000] [--Ns 1,2,4,8,16]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from fedsim_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--Ns", default="1,2,4,8,16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--products-only", action="store_true")
    a = ap.parse_args()
    K, P = a.K, a.P
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "librows_pieces.so"))
    lib.rows_pieces_f32.restype = ctypes.c_int
    lib.rows_pieces_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.slab_pieces_f32.restype = ctypes.c_int
    lib.slab_pieces_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(21)
    rows = [torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g) for _ in range(K)]
    table = ops.row_table(rows, dev)
    C = 4096
    Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
    for k in range(K):
        ops.pack_row(rows[k], Xb, k)
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    out = torch.empty(P, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def probe_rows(n):
        return lambda: lib.rows_pieces_f32(table.data_ptr(), w32.data_ptr(), K, P,
                                           out.data_ptr(), n, s)

    def probe_slab(n):
        return lambda: lib.slab_pieces_f32(Xb.data_ptr(), K, C, w32.data_ptr(), K, P,
                                           out.data_ptr(), n, s)

    variants = []
    for n in ([] if a.products_only else [int(x) for x in a.Ns.split(",")]):
        variants += [(f"probe_rows_N{n}", probe_rows(n), True), (f"probe_slab_N{n}", probe_slab(n), True)]
    def product_rows():
        ops.reduce_rows(rows, w32, out, table=table, checked=True, flags=ops.FEDAGG_NT)
        return 0

    def product_slab():
        ops.reduce_blocked(Xb, w32, out, flags=ops.FEDAGG_NT)
        return 0

    def product_rows_map(m, u=0):
        def f():
            ops.reduce_rows(rows, w32, out, table=table, checked=True,
                            flags=ops.FEDAGG_NT | ops.tuning_flags(mapping=m, unroll=u))
            return 0
        return f

    variants += [("product_rows_nt", product_rows, False), ("product_slab_nt", product_slab, False)]
    variants += [(f"product_rows_nt_{m}_u{u}", product_rows_map(m, u), False)
                 for m, u in (("narrow4", 8), ("narrow4", 16), ("narrow2", 16), ("wide", 0))]
    times = {n: [] for n, _, _ in variants}
    ref, ok = None, {}
    for r in range(a.rounds):
        for name, fn, is_probe in variants:
            if r == 0:
                rc = fn()
                assert not rc, (name, rc)
                torch.cuda.synchronize()
                if is_probe:
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
    for name, _, _ in variants:
        ms = float(np.median(times[name]))
        print(json.dumps(dict(K=K, P=P, variant=name, ms_median=ms,
                              GBps=(4.0 * K * P + 4.0 * P) / ms / 1e6,
                              bitwise_vs_probe_rows_N1=ok.get(name))), flush=True)


if __name__ == "__main__":
    main()
