"""FedDF teacher layers of SimpleCNN2 (fedsim/models/simple_models.py:245-252)
at K stacked teachers, B = 64 samples, timed per launch with HIP events:
conv1 (3 -> 64, 5x5, 24x24), the pad / LRN / max-pool pass after it, conv2
(64 -> 64, 5x5, 12x12) and the pass after that (sliding channel window, and
FEDAGG_POOL_PLANES: the per-block kernels, "_planes"), and SimpleCNN's 2 x 2 /
padding-1 pool on the same planes ("pool_cnn").  Several libfedagg BUILD
variants can be given; each is its own ctypes handle, run interleaved in one
process, and every output is compared bitwise with the first library's.
The convolutions run both ways: the default kernel choice ("lds" for these
shapes) and FEDAGG_CONV_GATHER ("gather", the im2col-gather kernel).

python tools/ab_teacher_conv.py [lib.so ...] [--K 500] [--rounds 3] [--iters 5]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import _native, ops  # noqa: E402

ENTRIES = ("fedagg_teacher_conv2d_f32", "fedagg_pad_lrn_maxpool_f32")


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in ENTRIES:
        res, args = _native.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--K", type=int, default=500)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")  # torch's HIP runtime first
    paths = a.libs or [_native.LIB_PATH]
    libs = [load(p) for p in paths]
    dev = torch.device("cuda:0")
    K, M = a.K, a.M
    P = 1_085_668
    g = torch.Generator(device=dev).manual_seed(5)
    slab = torch.empty(K, P, device=dev).normal_(0.0, 0.05, generator=g)
    x0 = torch.empty(M, 3, 24, 24, device=dev).normal_(0.0, 1.0, generator=g)
    # parameters_to_vector offsets of SimpleCNN2
    c1w, c1b, c2w, c2b = 0, 4800, 4864, 4864 + 102400
    stream = ops._stream_ptr(dev)
    lrn = (4, 0.001 / 9, 0.75, 1.0)
    pool = (3, 3, 2, 2, 0, 0)

    def conv(lib, x, shared, C, H, W, w, b, gather=False):
        s = _native.Conv2dShape(M, C, H, W, 64, 5, 5, 1, 1, 2, 2, H, W)
        y = torch.empty(K, M, 64, H, W, device=dev)
        rc = lib.fedagg_teacher_conv2d_f32(x.data_ptr(), 0 if shared else M * C * H * W,
                                           slab.data_ptr(), P, w, b, K, ctypes.byref(s),
                                           y.data_ptr(), _native.FEDAGG_RELU
                                           | (_native.FEDAGG_CONV_GATHER if gather else 0), stream)
        ops.check(rc, "conv")
        return y

    def pad_pool(lib, x, planes=False, cnn=False):
        # cnn: SimpleCNN's pool after conv2 (max_pool2d(2, 2, padding 1), no
        # pad / LRN; simple_models.py:155-159), on the same 12 x 12 planes
        args = (ops.pool_args(x.shape, (0, 0, 0, 0), None, (2, 2, 2, 2, 1, 1), planes=planes)
                if cnn else ops.pool_args(x.shape, (0, 1, 0, 1), lrn, pool, planes=planes))
        oh, ow = ops.pool_output(args)
        y = torch.empty(*x.shape[:-2], oh, ow, device=dev)
        ops.check(lib.fedagg_pad_lrn_maxpool_f32(x.data_ptr(), ctypes.byref(args), y.data_ptr(),
                                                 stream), "pool")
        return y

    # layer inputs of the chain, produced once by the first library
    c1 = conv(libs[0], x0, True, 3, 24, 24, c1w, c1b)
    p1 = pad_pool(libs[0], c1)
    c2 = conv(libs[0], p1, False, 64, 12, 12, c2w, c2b)
    layers = {
        "conv1": (lambda lib: conv(lib, x0, True, 3, 24, 24, c1w, c1b),
                  2.0 * K * M * 64 * 576 * 75, 4.0 * (M * 3 * 576 + K * M * 64 * 576)),
        "pool1": (lambda lib: pad_pool(lib, c1), 0.0, 4.0 * K * M * 64 * (576 + 144)),
        "conv2": (lambda lib: conv(lib, p1, False, 64, 12, 12, c2w, c2b),
                  2.0 * K * M * 64 * 144 * 1600, 4.0 * 2 * K * M * 64 * 144),
        "conv1_gather": (lambda lib: conv(lib, x0, True, 3, 24, 24, c1w, c1b, True),
                         2.0 * K * M * 64 * 576 * 75, 4.0 * (M * 3 * 576 + K * M * 64 * 576)),
        "conv2_gather": (lambda lib: conv(lib, p1, False, 64, 12, 12, c2w, c2b, True),
                         2.0 * K * M * 64 * 144 * 1600, 4.0 * 2 * K * M * 64 * 144),
        "pool2": (lambda lib: pad_pool(lib, c2), 0.0, 4.0 * K * M * 64 * (144 + 36)),
        "pool1_planes": (lambda lib: pad_pool(lib, c1, True), 0.0, 4.0 * K * M * 64 * (576 + 144)),
        "pool2_planes": (lambda lib: pad_pool(lib, c2, True), 0.0, 4.0 * K * M * 64 * (144 + 36)),
        "pool_cnn": (lambda lib: pad_pool(lib, c2, cnn=True), 0.0, 4.0 * K * M * 64 * (144 + 49)),
        "pool_cnn_planes": (lambda lib: pad_pool(lib, c2, True, cnn=True), 0.0,
                            4.0 * K * M * 64 * (144 + 49)),
    }
    ref = {name: fn(libs[0]) for name, (fn, _, _) in layers.items()}
    for name in ("pool1", "pool2", "pool_cnn"):  # sliding window vs per-block kernels: same bits
        same = torch.equal(ref[name].view(torch.int32), ref[name + "_planes"].view(torch.int32))
        print(json.dumps({"check": f"{name} slide vs planes", "bitwise": same}), flush=True)
        assert same
    for name in ("conv1", "conv2"):  # the two chain orders agree normwise
        u, v = ref[name].double(), ref[name + "_gather"].double()
        rel = ((u - v).norm() / v.norm()).item()
        print(json.dumps({"check": f"{name} lds vs gather", "rel_l2": rel}), flush=True)
        assert rel < 1e-5, rel
    torch.cuda.synchronize()
    times = {(p, n): [] for p in paths for n in layers}
    for _ in range(a.rounds):
        for path, lib in zip(paths, libs):
            for name, (fn, _, _) in layers.items():
                fn(lib)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(a.iters):
                    out = fn(lib)
                ev[1].record()
                torch.cuda.synchronize()
                times[(path, name)].append(ev[0].elapsed_time(ev[1]) / a.iters)
                if not torch.equal(out, ref[name]):
                    diff = (out - ref[name]).abs().max().item()
                    print(f"# {os.path.basename(path)} {name}: differs from the first library "
                          f"(max |diff| {diff:.3g})", file=sys.stderr)
    for path in paths:
        for name, (_, flop, byt) in layers.items():
            ms = min(times[(path, name)])
            rec = {"lib": os.path.basename(path), "layer": name, "K": K, "M": M, "ms": ms,
                   "all_ms": times[(path, name)]}
            if flop:
                rec["tflops"] = flop / ms / 1e9
                rec["frac_f32_mfma_peak"] = rec["tflops"] / 157.3
            rec["gbps"] = byt / ms / 1e6
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
