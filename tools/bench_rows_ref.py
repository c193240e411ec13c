"""fedagg_reduce_rows_ref (the dtype-generic keys' kernel) alone, against the
fp32 row-pointer kernel (fedagg_reduce_rows_f32) on the same bytes, for two
placements of the K client rows in HBM:

  distinct    K separate allocations (handed-over client tensors)
  contiguous  the K rows of one [K, P] tensor

K rows of 50 MB each (bf16 / fp16 P = 25 M, fp32 12.5 M, fp64 6.25 M), one
launch per timing (HIP events on the launch stream), best and median of
--reps; GB/s of client bytes read.

python tools/bench_rows_ref.py [--K 200] [--row-mb 50] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def timed(fn, reps):
    ts = []
    st = torch.cuda.current_stream()
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = ts[1:]  # the first launch pays the module load / table upload
    return min(ts), statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--row-mb", type=int, default=50)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dtypes", default="bfloat16,float16,float64,float32")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    for name in a.dtypes.split(","):
        dt = getattr(torch, name)
        esize = torch.empty((), dtype=dt).element_size()
        P = a.row_mb * 1_000_000 // esize
        nbytes = a.K * P * esize
        w = [float(50 + (k * 37) % 551) for k in range(a.K)]
        for layout in ("distinct", "contiguous"):
            g = torch.Generator(device=dev).manual_seed(3)
            if layout == "distinct":
                rows = [torch.empty(P, device=dev, dtype=torch.float32).normal_(0, 0.05, generator=g).to(dt)
                        for _ in range(a.K)]
            else:
                X = torch.empty(a.K, P, device=dev, dtype=dt)
                for k in range(a.K):
                    X[k].copy_(torch.empty(P, device=dev, dtype=torch.float32).normal_(0, 0.05, generator=g))
                rows = [X[k] for k in range(a.K)]
            out = torch.empty(P, device=dev, dtype=dt)
            if dt == torch.float32:
                w32 = torch.tensor([ops.fl32(x) for x in w], dtype=torch.float32, device=dev)
                table = ops.row_table(rows, dev)

                def fn():
                    ops.reduce_rows(rows, w32, out, table=table, checked=True)
            else:
                def fn():
                    ops.reduce_rows_ref(rows, w, out)
            best, med = timed(fn, a.reps)
            print(json.dumps(dict(dtype=name, layout=layout, K=a.K, P=P, ms_best=round(best, 3),
                                  ms_median=round(med, 3), gbps_best=round(nbytes / best / 1e6, 1),
                                  gbps_median=round(nbytes / med / 1e6, 1))), flush=True)
            del rows, out
            if layout == "contiguous":
                del X
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
