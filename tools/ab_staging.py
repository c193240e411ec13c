"""A/B of the ingest worker's staging copy (aggregators._STAGE_COPY: torch's
copy_ vs N memmove threads), interleaved in one process on the same box:
the bench's H2D-inclusive round (K=64 x 25 M, pageable and pinned) and a
config-2 host round (K=10 x 1 085 668 handed-over pageable vectors, add x K
+ get_sum, wall clock).

python tools/ab_staging.py [--variants torch,memmove4,memmove1] [--rounds 3]
(',' or ':' separate the variants; a variant "memmove4+zc" also reads the
staging slot in place, aggregators._HOST_PACK = "zero_copy")
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fedsim_amd.utils import SerialAggregator  # noqa: E402
from fedsim_amd.utils import aggregators as A  # noqa: E402


class _Rk(object):
    dev = torch.device("cuda:0")


def cfg2_round(vecs, reps=20):
    ts = []
    for _ in range(reps):
        agg = SerialAggregator(borrow_host=True, expected_rows=len(vecs))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, v in enumerate(vecs):
            agg.add("p", v, 1 + k)
        agg.get_sum("p")
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="torch,memmove4,memmove1")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--P", default="25000000", help="sizes of the H2D-inclusive leg, comma-separated")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    vecs = [torch.randn(1_085_668) for _ in range(10)]
    for r in range(a.rounds):
        for v in a.variants.replace(":", ",").split(","):
            A._STAGE_COPY, zc = v.split("+")[0], v.endswith("+zc")
            A._HOST_PACK = "zero_copy" if zc else "auto"
            for P in (int(x) for x in a.P.split(",")):
                h = bench.h2d_inclusive_leg(_Rk(), P)
                print(json.dumps({"round": r, "variant": v, "P": P, "h2d_pageable": h["pageable"],
                                  "h2d_pinned": h["pinned"], "ceiling": h["ceiling"],
                                  "checked": h["checked"]}), flush=True)
            print(json.dumps({"round": r, "variant": v,
                              "cfg2_K10_ms": round(cfg2_round(vecs), 3)}), flush=True)


if __name__ == "__main__":
    main()
