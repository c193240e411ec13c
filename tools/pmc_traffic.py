"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch
of the reduce kernel, with the gfx950 corrections from MI355X_MICROARCH.md §HBM:
  * counters are in KiB  -> x 1024
  * FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
    streaming read on gfx950 -> x 2 (k_reduce_vec's loads are dwordx4)
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
  * other widths are uncalibrated in the guide: with --calib DIR (a
    FETCH_SIZE / WRITE_SIZE pass over tools/pmc_calib, known 8 GiB per launch
    at 4 / 8 / 16 B per lane) the factors for --width are measured instead.
Writes profiles/pmc_traffic.json, read by bench.py for roofline.traffic.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --K 1000 --P 25000000
           [--kernel-match 'k_reduce_narrow<8, 2,'] [--label 'k_reduce_narrow<U=8, VW=2>']
           [--width 2 --calib-fetch DIR --calib-write DIR] [--step fused|split]
  fused: the reduce kernel with the server-step epilogue (EpiStep): algorithmic
         bytes 4KP + 4K + 12P (rows, weights, cloud read + write, grad write)
  split: the plain reduce (EpiStore): 4KP + 4K + 4P (the average's write)
"""
import argparse
import csv
import datetime
import glob
import hashlib
import json
import os
import socket

KERNEL = "k_reduce_vec"


def read_counter(d, name, match, tag=""):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if match in kn and tag in kn and row.get("Counter_Name") == name:
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for {match} in {files}")
    return vals


def lib_md5(path):
    """md5 of the profiled libfedagg.so: bench.py reports this summary's
    traffic only for the same build (bench.load_pmc)."""
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def gpu_name(d):
    """Agent name / id rocprofv3 recorded next to the counters, if any."""
    for fn in glob.glob(os.path.join(d, "**", "*agent_info.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Agent_Type", row.get("Type", "")).upper().endswith("GPU"):
                    return "%s (%s)" % (row.get("Marketing_Name", row.get("Name", "?")),
                                        row.get("Name", "?"))
    return None


CALIB_BYTES = 8 << 30  # tools/pmc_calib.hip: bytes read / written per launch


def calib_factor(d, name, kernel, width):
    """Bytes per counted byte for `width`-dword accesses, from tools/pmc_calib."""
    vals = read_counter(d, name, f"{kernel}<{width}>")
    return CALIB_BYTES / (sum(vals) / len(vals) * 1024)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--K", type=int, required=True)
    ap.add_argument("--P", type=int, required=True)
    ap.add_argument("--layout", default="blocked4096", help="strided | blocked<C>")
    ap.add_argument("--step", default="fused", choices=["fused", "split"])
    ap.add_argument("--kernel-match", default=KERNEL,
                    help="substring of the measured kernel's name in the counter CSV")
    ap.add_argument("--label", default=KERNEL, help="kernel name bench.py matches on")
    ap.add_argument("--width", type=int, default=4, choices=[1, 2, 4],
                    help="dwords per lane of the kernel's client-row loads / result stores")
    ap.add_argument("--calib-fetch", default=None)
    ap.add_argument("--calib-write", default=None)
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(__file__), "..", "fedsim_amd",
                                                  "libfedagg.so"),
                    help="the library the profiled bench loaded (its md5 is the build id)")
    ap.add_argument("--profile", default=None,
                    help="where the summary is committed (profiles/<round>/), for provenance")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                  "pmc_traffic.json"))
    a = ap.parse_args()
    tag = "EpiStep" if a.step == "fused" else "EpiStore"
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE", a.kernel_match, tag)
    write = read_counter(a.write_dir, "WRITE_SIZE", a.kernel_match, tag)
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    calib = {}
    if a.calib_fetch:
        calib["fetch"] = {w: calib_factor(a.calib_fetch, "FETCH_SIZE", "calib_read", w)
                          for w in (1, 2, 4)}
    if a.calib_write:
        calib["write"] = {w: calib_factor(a.calib_write, "WRITE_SIZE", "calib_write", w)
                          for w in (1, 2, 4)}
    f_fac = calib["fetch"][a.width] if "fetch" in calib else 2.0
    w_fac = calib["write"][a.width] if "write" in calib else 1.0
    fetch_b = f_kib * 1024 * f_fac
    write_b = w_kib * 1024 * w_fac
    alg = 4.0 * a.K * a.P + 4.0 * a.K + (12.0 if a.step == "fused" else 4.0) * a.P
    out = dict(
        kernel=a.label, epilogue=tag, K=a.K, P=a.P, layout=a.layout, step=a.step,
        width_dwords=a.width, fetch_factor=f_fac, write_factor=w_fac, calibration=calib,
        dispatches=dict(fetch=len(fetch), write=len(write)),
        FETCH_SIZE_KiB_mean=f_kib, WRITE_SIZE_KiB_mean=w_kib,
        fetch_bytes_corrected=fetch_b, write_bytes=write_b,
        hbm_bytes_per_launch=fetch_b + write_b,
        alg_bytes_per_launch=alg,
        traffic_over_alg=(fetch_b + write_b) / alg,
        source=dict(
            lib_md5=lib_md5(a.lib),
            profile=a.profile or os.path.relpath(os.path.abspath(a.fetch_dir)),
            fetch_dir=a.fetch_dir, write_dir=a.write_dir,
            host=socket.gethostname(), gpu=gpu_name(a.fetch_dir),
            utc=datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        ),
        corrections=("KiB->B x1024; FETCH_SIZE x fetch_factor, WRITE_SIZE x write_factor: "
                     "measured on tools/pmc_calib (known 8 GiB at this width)" if calib else
                     "KiB->B x1024; FETCH_SIZE x2 for 16B/lane streaming reads on gfx950 "
                     "(MI355X_MICROARCH.md §HBM)"),
    )
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
