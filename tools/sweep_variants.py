"""A/B of libfedagg BUILD variants (compile-time knobs: FEDAGG_ROLL,
FEDAGG_WAVES_PER_EU, ...) on the headline fused round, interleaved in one
process so box-to-box spread cancels.  Each variant is its own .so loaded with
its own ctypes handle; outputs are checked bitwise against the first variant.

python tools/sweep_variants.py tools/variants/libfedagg_base.so tools/variants/libfedagg_roll.so
    [--K 1000] [--P 25000000] [--rounds 3] [--iters 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import _native, ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in ("fedagg_reduce_step_blocked_f32", "fedagg_reduce_blocked_f32"):
        res, args = _native.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--C", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant-flags", default="",
                    help="comma-separated extra flag words, one per library (tuning bits "
                         "OR'ed into the fused call, e.g. ops.tuning_flags(unroll=16))")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--shape", default="", help="also time tools/shape_kernel.hip's probe .so")
    ap.add_argument("--fill", default="normal", choices=["normal", "const"],
                    help="slab contents: N(0, 0.05) floats, or one constant word "
                         "(data-dependent power check)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K, P, C = a.K, a.P, a.C
    Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    for b0 in range(0, Xb.shape[0], 256):
        if a.fill == "const":
            Xb[b0:b0 + 256].fill_(0.75)
        else:
            Xb[b0:b0 + 256].normal_(0.0, 0.05, generator=g)
    w = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
    W32 = ops.fl32(sum(w))
    libs = [load(p) for p in a.libs]
    vflags = [int(v, 0) for v in a.variant_flags.split(",")] if a.variant_flags else []
    vflags += [0] * (len(libs) - len(vflags))
    stream = torch.cuda.current_stream(dev).cuda_stream
    cloud0 = torch.zeros(P, device=dev)
    results = {i: [] for i in range(len(a.libs))}
    outs = {}
    alg = 4.0 * K * P + 4.0 * K + 12.0 * P
    for r in range(a.rounds):
        for i, (path, lib, xf) in enumerate(zip(a.libs, libs, vflags)):
            cloud = cloud0.clone()
            grad = torch.empty(P, device=dev)
            step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)

            def run():
                rc = lib.fedagg_reduce_step_blocked_f32(
                    Xb.data_ptr(), K, C, w32.data_ptr(), K, P, None, W32, 0x1 | 0x2 | xf,
                    ctypes.byref(step.args), stream)
                assert rc == 0, rc

            run()
            torch.cuda.synchronize()
            if r == 0:
                outs[i] = cloud.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            results[i].append(ms)
    # the plain reduce (no server step) of the first library: buffer-descriptor
    # loads (default) vs flat global loads (FEDAGG_FLAT), same slab
    avg = torch.empty(P, device=dev)
    lib0 = libs[0]
    flat_res = {}
    for r in range(a.rounds):
        for name, extra in (("reduce_buffer", 0), ("reduce_flat", _native.FEDAGG_FLAT)):
            flags = 0x1 | 0x2 | ops.default_flags(C) | extra

            def run():
                rc = lib0.fedagg_reduce_blocked_f32(Xb.data_ptr(), K, C, w32.data_ptr(), K, P,
                                                    None, avg.data_ptr(), W32, flags, stream)
                assert rc == 0, rc

            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            flat_res.setdefault(name, []).append(e0.elapsed_time(e1) / a.iters)
    for name, v in flat_res.items():
        ms = min(v)
        print(json.dumps(dict(lib=os.path.basename(a.libs[0]), kernel=name, ms_min=ms,
                              GBps=(4.0 * K * P + 4.0 * K + 4.0 * P) / ms / 1e6)), flush=True)
    if a.shape:
        shp = ctypes.CDLL(os.path.abspath(a.shape), mode=ctypes.RTLD_LOCAL)
        shp.shape_reduce.restype = ctypes.c_int
        shp.shape_reduce.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        sink = torch.zeros(1, device=dev)
        ts = []
        for r in range(a.rounds):
            def run():
                assert shp.shape_reduce(Xb.data_ptr(), K, K, Xb.shape[0], w32.data_ptr(),
                                        sink.data_ptr(), stream) == 0

            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / a.iters)
        print(json.dumps(dict(lib=os.path.basename(a.shape), kernel="shape (checksum only)",
                              ms_min=min(ts), GBps=4.0 * K * Xb.shape[0] * C / min(ts) / 1e6)),
              flush=True)
    ref = outs[0]
    for i, path in enumerate(a.libs):
        ms = min(results[i])
        print(json.dumps(dict(lib=os.path.basename(path), flags=vflags[i], ms_min=ms,
                              ms_median=float(np.median(results[i])),
                              ms_all=[round(x, 4) for x in results[i]],
                              GBps=alg / ms / 1e6,
                              bitwise_vs_first=bool(torch.equal(outs[i].view(torch.int32),
                                                                ref.view(torch.int32))))),
              flush=True)


if __name__ == "__main__":
    main()
