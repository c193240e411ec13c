"""HBM traffic of the FedDF teacher kernels from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes over tools/ab_teacher_conv.py (SimpleCNN2 layers, K=500,
B=64; tools/gpu_run.sh (pmc / sq steps; the round-2 script is in git history)), corrected by the per-box calibration passes
over tools/pmc_calib (8 GiB read / written once per kernel, so factor =
8 GiB / counter bytes; MI355X_MICROARCH.md: counters in KiB, FETCH_SIZE
half of a streaming read on gfx950).  Algorithmic bytes per launch: the
layer's input read once and its output written once.

python tools/pmc_teachers.py gpurun_out/r02pmc [run prefix, default "teach"] \
    > profiles/r02pmc/teacher_traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys

K, M = 500, 64
ALG = {  # kernel name prefix -> (label, algorithmic read bytes, write bytes)
    "k_pad_lrn_maxpool_slide<4, 3, 8>": ("pool1 (sliding window)", 4.0 * K * M * 64 * 576, 4.0 * K * M * 64 * 144),
    "k_pad_lrn_maxpool_q<4, 3>": ("pool1 (per-block planes)", 4.0 * K * M * 64 * 576, 4.0 * K * M * 64 * 144),
    "k_pad_lrn_maxpool_slide<4, 1, 16>": ("pool2 (sliding window)", 4.0 * K * M * 64 * 144, 4.0 * K * M * 64 * 36),
    "k_pad_lrn_maxpool_q<4, 1>": ("pool2 (per-block planes)", 4.0 * K * M * 64 * 144, 4.0 * K * M * 64 * 36),
    "k_teacher_conv2d_flat<5, 3, 16,": ("conv1 (flat, LDS)", 4.0 * (M * 3 * 576 + K * 64 * 76), 4.0 * K * M * 64 * 576),
    "k_teacher_conv2d_lds<5, 4, 8>": ("conv2 (chunked, LDS)", 4.0 * (K * M * 64 * 144 + K * 64 * 1601), 4.0 * K * M * 64 * 144),
}


def per_dispatch(d, counter):
    out = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(d, "*counter_collection.csv")):
        acc, names = collections.defaultdict(float), {}
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] == counter:
                acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for k, v in acc.items():
            out[names[k]].append(v * 1024.0)
    return out


def factor(d, counter, kernel):
    vals = [v for n, vs in per_dispatch(d, counter).items() if kernel in n for v in vs]
    return (8 << 30) / (sum(vals) / len(vals))


def main():
    root = sys.argv[1]
    run = sys.argv[2] if len(sys.argv) > 2 else "teach"
    ff = factor(os.path.join(root, "calib_fetch"), "FETCH_SIZE", "calib_read<1>")
    fw = factor(os.path.join(root, "calib_write"), "WRITE_SIZE", "calib_write<1>")
    fetch = per_dispatch(os.path.join(root, run + "_fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(root, run + "_write"), "WRITE_SIZE")
    rows = []
    for prefix, (label, ar, aw) in ALG.items():
        fv = [v for n, vs in fetch.items() if prefix in n for v in vs]
        wv = [v for n, vs in write.items() if prefix in n for v in vs]
        if not fv or not wv:
            continue
        r = sum(fv) / len(fv) * ff
        w = sum(wv) / len(wv) * fw
        rows.append(dict(kernel=prefix, layer=label, hbm_read_bytes=r, hbm_write_bytes=w,
                         alg_read_bytes=ar, alg_write_bytes=aw, read_over_alg=r / ar,
                         write_over_alg=w / aw, launches=len(fv)))
    print(json.dumps(dict(K=K, M=M, run=run, fetch_factor_4B=ff, write_factor_4B=fw, kernels=rows),
                     indent=1))


if __name__ == "__main__":
    main()
