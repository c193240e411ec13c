"""HBM bytes per launch of the wide-tile row kernels (k_reduce_rows_ref:
bf16 / fp16 / fp64 generic keys, and RefF32 for fedagg_reduce_rows_f32's
borrowed rows) from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over
tools/bench_rows_ref.py (K rows of ROW_MB each, every launch the same size),
against the algorithmic bytes: K rows read once + the sum written once.
Corrections as tools/pmc_traffic.py: KiB -> B, and the per-width factors
measured on tools/pmc_calib (every load / store of these kernels is 16 B per
lane).

python tools/pmc_rows_tiles.py FETCH_DIR WRITE_DIR --calib-fetch DIR --calib-write DIR
       [--K 200] [--row-mb 50] [--out profiles/r05aa/pmc_rows_tiles.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import calib_factor  # noqa: E402

ESIZE = {"RefBf16": 2, "RefF16": 2, "RefF64": 8, "RefF32": 4}


def per_kernel(d, counter):
    out = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if "k_reduce_rows_ref" not in kn or row.get("Counter_Name") != counter:
                    continue
                m = re.search(r"k_reduce_rows_ref<\(anonymous namespace\)::(\w+), (\d+), (\d+), (\d+)>", kn)
                if not m or m.group(2) == "1":  # the scalar tail launches
                    continue
                key = f"{m.group(1)} VW={m.group(2)} U={m.group(3)} NV={m.group(4)}"
                out.setdefault(key, []).append(float(row["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--row-mb", type=float, default=50)
    ap.add_argument("--out")
    a = ap.parse_args()
    f_fac = calib_factor(a.calib_fetch, "FETCH_SIZE", "calib_read", 4)
    w_fac = calib_factor(a.calib_write, "WRITE_SIZE", "calib_write", 4)
    fetch, write = per_kernel(a.fetch, "FETCH_SIZE"), per_kernel(a.write, "WRITE_SIZE")
    res = dict(K=a.K, row_bytes=int(a.row_mb * 1e6), fetch_factor=f_fac, write_factor=w_fac,
               kernels={})
    for key in sorted(fetch):
        es = ESIZE[key.split()[0]]
        P = int(a.row_mb * 1e6) // es
        alg_read, alg_write = a.K * P * es, P * es
        fb = statistics.median(fetch[key]) * 1024 * f_fac
        wb = statistics.median(write.get(key, [float("nan")])) * 1024 * w_fac
        res["kernels"][key] = dict(dispatches=len(fetch[key]), P=P, fetch_bytes=fb,
                                   write_bytes=wb, alg_read=alg_read, alg_write=alg_write,
                                   read_over_alg=fb / alg_read, write_over_alg=wb / alg_write,
                                   traffic_over_alg=(fb + wb) / (alg_read + alg_write))
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
