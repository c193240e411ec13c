"""Config 5's per-GPU stream (P = 125 M columns, clients re-read from a resident
column-blocked pool of `pool` rows, chained through acc_in pass after pass)
against the pool size and the column mapping.  Each timed unit reduces 1000
client rows (1000 / pool passes), so every line moves the same algorithmic
bytes; chaining adds 8 P bytes per extra pass.  Every variant is checked
bitwise against the first of its pool size.

python tools/ab_cfg5_pool.py [--P 125000000] [--pools 50,100,200,250]
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
    ap.add_argument("--P", type=int, default=125_000_000)
    ap.add_argument("--rows", type=int, default=1000, help="client rows per timed unit")
    ap.add_argument("--pools", default="50,100,200,250")
    ap.add_argument("--mappings", default="auto,narrow2,narrow4,wide")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    P = a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    C = ops.choose_block_cols(P)
    acc = torch.empty(P, device=dev)
    for pool in [int(x) for x in a.pools.split(",")]:
        passes = a.rows // pool
        Xb = torch.empty(ops.blocked_shape(pool, P, C), device=dev).normal_(0, 0.05, generator=g)
        w32 = torch.randint(50, 601, (pool,), device=dev).float()
        maps = a.mappings.split(",")
        ref, times = None, {m: [] for m in maps}
        ok = {}
        for r in range(a.rounds):
            for m in maps:
                f = ops.default_flags(C) | ops.tuning_flags(mapping=m)

                def unit():
                    for i in range(passes):
                        ops.reduce_blocked(Xb, w32, acc, acc_in=None if i == 0 else acc, flags=f)

                if r == 0:
                    unit()
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = acc.clone()
                    ok[m] = bool(torch.equal(acc.view(torch.int32), ref.view(torch.int32)))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                unit()
                e1.record()
                torch.cuda.synchronize()
                times[m].append(e0.elapsed_time(e1))
        for m in maps:
            ms = float(np.median(times[m]))
            print(json.dumps(dict(P=P, C=C, pool=pool, passes=passes, mapping=m,
                                  resolved=ops.column_mapping(P, ops.tuning_flags(mapping=m), B=pool),
                                  ms_median=ms, GBps=4.0 * passes * pool * P / ms / 1e6,
                                  bitwise_vs_first=ok[m])), flush=True)
        del Xb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
