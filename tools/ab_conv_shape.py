"""One teacher Conv2d shape across libfedagg BUILD variants: K stacked
teachers, M = 64 images, timed per launch with HIP events, rounds
interleaved, every output compared with the first library's (normwise when
the variants' chain orders differ, see fedagg_conv_order).

Default shape: SimpleCNN's conv2 (fedsim/models/simple_models.py:112-118:
32 -> 64 channels, 5 x 5, padding 1, on the 14 x 14 pooled conv1 output).

python tools/ab_conv_shape.py lib_a.so [lib_b.so ...] [--K 500] [--C 32] [--H 14]
       [--OC 64] [--ks 5] [--pad 1] [--shared] [--pool-pad 0|1]

--shared: one input for every teacher (a model's first layer); --pool-pad: the
2 x 2 / 2 max pool fused into the store (FEDAGG_CONV_MAXPOOL2).  SimpleCNN's
conv1 + pool: --C 1 --H 28 --OC 32 --pad 1 --shared --pool-pad 1.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import _native, ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in ("fedagg_teacher_conv2d_f32", "fedagg_conv_order"):
        res, args = _native.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--K", type=int, default=500)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--C", type=int, default=32)
    ap.add_argument("--H", type=int, default=14)
    ap.add_argument("--OC", type=int, default=64)
    ap.add_argument("--ks", type=int, default=5)
    ap.add_argument("--pad", type=int, default=1)
    ap.add_argument("--shared", action="store_true")
    ap.add_argument("--pool-pad", type=int, default=-1)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")  # torch's HIP runtime first
    libs = [load(p) for p in a.libs]
    dev = torch.device("cuda:0")
    K, M, C, H, OC, ks, pad = a.K, a.M, a.C, a.H, a.OC, a.ks, a.pad
    OH = H + 2 * pad - ks + 1
    R = C * ks * ks
    P = OC * R + OC
    g = torch.Generator(device=dev).manual_seed(5)
    slab = torch.empty(K, P, device=dev).normal_(0.0, 0.05, generator=g)
    x = torch.empty(1 if a.shared else K, M, C, H, H, device=dev).normal_(0.0, 1.0,
                                                                          generator=g).relu_()
    flags = _native.FEDAGG_RELU
    OP = OH
    if a.pool_pad >= 0:
        flags |= _native.FEDAGG_CONV_MAXPOOL2 | (_native.FEDAGG_CONV_POOL_PAD1 if a.pool_pad else 0)
        OP = (OH + 2 * a.pool_pad - 2) // 2 + 1
    s = _native.Conv2dShape(M, C, H, H, OC, ks, ks, 1, 1, pad, pad, OH, OH)
    stream = ops._stream_ptr(dev)

    def conv(lib):
        y = torch.empty(K, M, OC, OP, OP, device=dev)
        ops.check(lib.fedagg_teacher_conv2d_f32(x.data_ptr(), 0 if a.shared else M * C * H * H,
                                                slab.data_ptr(), P, 0, OC * R, K, ctypes.byref(s),
                                                y.data_ptr(), flags, stream), "conv")
        return y

    ref = conv(libs[0])
    times = {p: [] for p in a.libs}
    for _ in range(a.rounds):
        for path, lib in zip(a.libs, libs):
            conv(lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                y = conv(lib)
            e1.record()
            torch.cuda.synchronize()
            times[path].append(e0.elapsed_time(e1) / a.iters)
            times.setdefault((path, "rel"), (y.double() - ref.double()).norm().item()
                             / ref.double().norm().item())
            times.setdefault((path, "bitwise"), torch.equal(y.view(torch.int32),
                                                            ref.view(torch.int32)))
    flop = 2.0 * K * M * OH * OH * OC * R
    for path, lib in zip(a.libs, libs):
        ms = min(times[path])
        print(json.dumps(dict(lib=os.path.basename(path), K=K, M=M, C=C, H=H, OC=OC, ks=ks,
                              pool_pad=a.pool_pad, shared=a.shared,
                              order=lib.fedagg_conv_order(ctypes.byref(s), 0), ms=ms,
                              all_ms=times[path], tflops=flop / ms / 1e9,
                              frac_f32_mfma_peak=flop / ms / 1e9 / 157.3,
                              rel_l2_vs_first=times[(path, "rel")],
                              bitwise_vs_first=times[(path, "bitwise")])), flush=True)


if __name__ == "__main__":
    main()
