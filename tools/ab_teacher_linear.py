"""One teacher Linear shape across libfedagg BUILD variants: K stacked
teachers, M = 64 samples, per-teacher inputs (every layer after the first),
timed per launch with HIP events after warm-up launches, rounds interleaved
with the order rotated each round, every output compared
bit for bit with the first library's.

Default shape: SimpleCNN's fc (fedsim/models/simple_models.py:119-121:
3136 -> 512, the wide, weight-streaming layer).

python tools/ab_teacher_linear.py lib_a.so [lib_b.so ...] [--K 500] [--inf 3136] [--out 512]
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
    res, args = _native.SIGNATURES["fedagg_teacher_linear_f32"]
    fn = lib.fedagg_teacher_linear_f32
    fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--K", type=int, default=500)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--inf", type=int, default=3136)
    ap.add_argument("--out", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warm", type=int, default=20)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")  # torch's HIP runtime first
    libs = [load(p) for p in a.libs]
    dev = torch.device("cuda:0")
    K, M, IN, OUT = a.K, a.M, a.inf, a.out
    P = (IN * OUT + OUT + 3) // 4 * 4  # rows 16-byte aligned, as TeacherEnsemble pads them
    g = torch.Generator(device=dev).manual_seed(5)
    slab = torch.empty(K, P, device=dev).normal_(0.0, 0.02, generator=g)
    x = torch.empty(K, M, IN, device=dev).normal_(0.0, 1.0, generator=g).relu_()
    stream = ops._stream_ptr(dev)

    def linear(lib):
        y = torch.empty(K, M, OUT, device=dev)
        ops.check(lib.fedagg_teacher_linear_f32(x.data_ptr(), M * IN, slab.data_ptr(), P, 0,
                                                IN * OUT, K, M, IN, OUT, y.data_ptr(),
                                                _native.FEDAGG_RELU, stream), "linear")
        return y

    ref = linear(libs[0])
    for _ in range(a.warm):  # clocks up before the first timed round
        for lib in libs:
            linear(lib)
    torch.cuda.synchronize()
    times = {p: [] for p in a.libs}
    same = {}
    pairs = list(zip(a.libs, libs))
    for rnd in range(a.rounds):
        # each round starts with the next library: no variant always runs
        # first (or last) in its round
        for path, lib in pairs[rnd % len(pairs):] + pairs[:rnd % len(pairs)]:
            linear(lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                y = linear(lib)
            e1.record()
            torch.cuda.synchronize()
            times[path].append(e0.elapsed_time(e1) / a.iters)
            same.setdefault(path, torch.equal(y.view(torch.int32), ref.view(torch.int32)))
    flop = 2.0 * K * M * IN * OUT
    for path in a.libs:
        ms = min(times[path])
        print(json.dumps(dict(lib=os.path.basename(path), K=K, M=M, inf=IN, out=OUT, ms=ms,
                              all_ms=times[path], tflops=flop / ms / 1e9,
                              frac_f32_mfma_peak=flop / ms / 1e9 / 157.3,
                              bitwise_vs_first=same[path])), flush=True)


if __name__ == "__main__":
    main()
