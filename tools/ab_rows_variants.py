"""A/B of libfedagg BUILD variants on the borrowed-row round (K separate
client tensors, pointer table): fused FedAvg step (fedagg_reduce_step_rows_f32)
and the plain reduce (fedagg_reduce_rows_f32), interleaved in one process;
outputs checked bitwise against the first library.

python tools/ab_rows_variants.py fedsim_amd/libfedagg.so tools/variants/libfedagg_x.so
    [--K 1000] [--P 25000000] [--rounds 5]
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

FNS = ("fedagg_reduce_step_rows_f32", "fedagg_reduce_rows_f32")


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name in FNS:
        res, args = _native.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(13)
    rows = [torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g) for _ in range(K)]
    table = ops.row_table(rows, dev)
    w = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
    W32 = ops.fl32(sum(w))
    libs = [load(p) for p in a.libs]
    stream = torch.cuda.current_stream(dev).cuda_stream
    cloud0 = torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g)
    cloud = torch.empty(P, device=dev)
    grad = torch.empty(P, device=dev)
    avg = torch.empty(P, device=dev)
    step = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)
    fl = 0x1 | 0x2 | ops.FEDAGG_NT
    times = {(i, kind): [] for i in range(len(libs)) for kind in ("step", "reduce")}
    ref = {}
    for r in range(a.rounds):
        for i, lib in enumerate(libs):
            for kind in ("step", "reduce"):
                if kind == "step":
                    def run():
                        rc = lib.fedagg_reduce_step_rows_f32(table.data_ptr(), w32.data_ptr(), K,
                                                             P, None, W32, fl,
                                                             ctypes.byref(step.args), stream)
                        assert rc == 0, rc
                    out = cloud
                    cloud.copy_(cloud0)
                else:
                    def run():
                        rc = lib.fedagg_reduce_rows_f32(table.data_ptr(), w32.data_ptr(), K, P,
                                                        None, avg.data_ptr(), W32, fl, stream)
                        assert rc == 0, rc
                    out = avg
                run()
                torch.cuda.synchronize()
                if r == 0:
                    if kind not in ref:
                        ref[kind] = out.clone()
                    assert torch.equal(out.view(torch.int32), ref[kind].view(torch.int32)), \
                        (a.libs[i], kind)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[(i, kind)].append(e0.elapsed_time(e1) / a.iters)
    for (i, kind), t in times.items():
        ms = float(np.median(t))
        alg = 4.0 * K * P + 4.0 * K + (12.0 if kind == "step" else 4.0) * P
        print(json.dumps(dict(lib=os.path.basename(a.libs[i]), kind=kind, K=K, P=P,
                              ms_median=ms, ms_min=float(np.min(t)), GBps=alg / ms / 1e6,
                              bitwise_vs_first=True)), flush=True)


if __name__ == "__main__":
    main()
