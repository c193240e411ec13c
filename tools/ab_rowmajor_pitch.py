"""Row-major client rows: does the row pitch (bytes between the starts of
consecutive client rows) move the exact reduce?  One [K, ldx] allocation per
pitch, ldx = P + pad floats, reduced by fedagg_reduce_f32 (the same access
shape as borrowed client tensors), against the column-blocked slab of the
same data; rounds interleaved, outputs compared bit for bit.

python tools/ab_rowmajor_pitch.py [--K 600] [--P 25000000] [--pads 0,256,1024,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=600)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--pads", default="0,64,256,1024,4096,16384,65536,262144")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    C = ops.choose_block_cols(P)
    Xb = torch.zeros(ops.blocked_shape(K, P, C), device=dev)
    src = torch.empty(P, device=dev)
    for k in range(K):
        src.normal_(0, 1, generator=g)
        ops.pack_row(src, Xb, k)
    w32 = torch.randint(50, 601, (K,), device=dev, generator=g).float()
    W = float(w32.sum().item())
    ref = torch.empty(P, device=dev)
    ops.reduce_blocked(Xb, w32, ref, W=W, flags=ops.default_flags(C))
    out = torch.empty(P, device=dev)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    res = {"blocked": [timed(lambda: ops.reduce_blocked(Xb, w32, out, W=W,
                                                        flags=ops.default_flags(C)))
                       for _ in range(a.rounds)]}
    for pad in [int(v) for v in a.pads.split(",")]:
        ldx = P + pad
        X = torch.empty((K, ldx), device=dev)
        for k in range(K):  # row k of the slab, unpacked from the blocked copy
            ops.unpack_row(Xb, k, P, out=X[k, :P])
        ts = [timed(lambda: ops.reduce_slab(X[:, :P], w32, out, W=W)) for _ in range(a.rounds)]
        assert torch.equal(out, ref), pad
        res[f"rowmajor_pad{pad}"] = ts
        del X
        torch.cuda.empty_cache()
    res["blocked_again"] = [timed(lambda: ops.reduce_blocked(Xb, w32, out, W=W,
                                                              flags=ops.default_flags(C)))
                            for _ in range(a.rounds)]
    for name, ts in res.items():
        ms = min(ts)
        print(json.dumps(dict(layout=name, K=K, P=P, ms=ms, all_ms=ts,
                              gbps=4.0 * K * P / ms / 1e6)), flush=True)


if __name__ == "__main__":
    main()
