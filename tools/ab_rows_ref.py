"""A/B of libfedagg BUILD variants of fedagg_reduce_rows_ref (the generic
keys' kernel; float32 in --dtypes: fedagg_reduce_rows_f32, the fp32 kernel's
borrowed-row path): bf16 / fp16 / fp64 rounds of K handed-over client rows (K
separate 50 MB allocations), each library its own ctypes handle, run
interleaved in one process, every output compared bitwise with the first
library's.  HIP events around each launch; GB/s of client bytes read.

  python tools/ab_rows_ref.py lib_a.so lib_b.so ... [--K 200] [--rounds 3] [--iters 5]

Variants are built with -DFEDAGG_REF_U / _NV / _STRIDE (fedagg_kernels.hip)
by ``--build OUTDIR NAME=-DX=1,-DY=2 ...`` (build container, CPU only).
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def build(outdir, specs):
    import __graft_entry__ as G
    os.makedirs(outdir, exist_ok=True)
    src = os.path.join(REPO, "fedsim_amd", "csrc", "fedagg_kernels.hip")
    from concurrent.futures import ThreadPoolExecutor

    def one(spec):
        name, _, defs = spec.partition("=")
        flags = [d for d in defs.split(",") if d]
        out = os.path.join(outdir, f"libfedagg_{name}.so")
        subprocess.check_call([G.HIPCC, *G.HIP_FLAGS, *flags, "-o", out, src])
        return out

    with ThreadPoolExecutor(4) as pool:  # ~3 GB of host memory per hipcc
        for out in pool.map(one, specs):
            print(out, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--build", nargs="+", metavar=("OUTDIR", "NAME=DEFS"))
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--row-mb", default="50", help="row sizes in MB, separated by : or ,")
    ap.add_argument("--odd", type=int, default=0, help="elements added to every P (tails)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dtypes", default="bfloat16,float16,float64")
    ap.add_argument("--f32-codes", default="",
                    help="float32: also run fedagg_reduce_rows_ref with these dtype codes "
                         "(builds with -DFEDAGG_EXP_F32REF), separated by :")
    a = ap.parse_args()
    if a.build:
        build(a.build[0], a.build[1:])
        return
    import torch
    from fedsim_amd import _native, ops

    torch.zeros(1, device="cuda")  # torch's HIP runtime first
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
        fns = {}
        for entry in ("fedagg_reduce_rows_ref", "fedagg_reduce_rows_f32"):
            res, args = _native.SIGNATURES[entry]
            fn = getattr(lib, entry)
            fn.restype, fn.argtypes = res, args
            fns[entry] = fn
        libs.append((os.path.basename(p), fns))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    codes = {torch.bfloat16: _native.FEDAGG_DTYPE_BF16, torch.float16: _native.FEDAGG_DTYPE_F16,
             torch.float64: _native.FEDAGG_DTYPE_F64}
    for name, mb in [(n, m) for m in a.row_mb.replace(":", ",").split(",") for n in a.dtypes.replace(":", ",").split(",")]:
        dt = getattr(torch, name)
        esize = torch.empty((), dtype=dt).element_size()
        P = int(float(mb) * 1_000_000) // esize + a.odd
        g = torch.Generator(device=dev).manual_seed(11)
        rows = [torch.empty(P, device=dev, dtype=torch.float32).normal_(0, 0.05, generator=g).to(dt)
                for _ in range(a.K)]
        wdt = torch.float64 if dt == torch.float64 else torch.float32
        w = torch.tensor([float(50 + (k * 37) % 551) for k in range(a.K)], dtype=wdt, device=dev)
        table = ops.row_table_from_ptrs([r.data_ptr() for r in rows], dev)
        variants = []
        for n, fns in libs:
            if dt == torch.float32:
                variants.append((n, lambda out, f=fns["fedagg_reduce_rows_f32"]: f(
                    table.data_ptr(), w.data_ptr(), a.K, P, None, out.data_ptr(), 0.0,
                    _native.FEDAGG_INIT, ops._stream_ptr(dev))))
                for code in [int(c) for c in a.f32_codes.replace(":", ",").split(",") if c]:
                    variants.append((f"{n}#{code}", lambda out, f=fns["fedagg_reduce_rows_ref"], c=code: f(
                        c, table.data_ptr(), w.data_ptr(), a.K, P, None, out.data_ptr(),
                        _native.FEDAGG_INIT, ops._stream_ptr(dev))))
            else:
                variants.append((n, lambda out, f=fns["fedagg_reduce_rows_ref"]: f(
                    codes[dt], table.data_ptr(), w.data_ptr(), a.K, P, None, out.data_ptr(),
                    _native.FEDAGG_INIT, ops._stream_ptr(dev))))
        outs = [torch.empty(P, device=dev, dtype=dt) for _ in variants]
        times = {n: [] for n, _ in variants}
        for _ in range(a.rounds):
            for (n, fn), out in zip(variants, outs):
                for it in range(a.iters + 1):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    rc = fn(out)
                    e1.record(st)
                    e1.synchronize()
                    if rc != 0:
                        raise RuntimeError(f"{n}: rc {rc}")
                    if it:
                        times[n].append(e0.elapsed_time(e1))
        ib = {torch.float64: torch.int64, torch.float32: torch.int32}.get(dt, torch.int16)
        for (n, _), out in zip(variants, outs):
            med = statistics.median(times[n])
            print(json.dumps(dict(lib=n, dtype=name, K=a.K, P=P, ms_median=round(med, 4),
                                  ms_best=round(min(times[n]), 4),
                                  gbps=round(a.K * P * esize / med / 1e6, 1),
                                  same_bits=bool(torch.equal(out.view(ib), outs[0].view(ib))))),
                  flush=True)
        del rows, outs, table
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
