"""Mismatch census of fedagg_reduce_rows_ref's all-scalar path (a row off
16-B alignment) against its vector path on the same rows, per dtype and P:
mismatch count, first indices and values (tests/test_generic_keys.py
test_reference_kernel_tile_rungs is the pass / fail form).

python tests/debug_rows_ref.py  (a GPU script, not collected by pytest; the
oracle is its checker)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402


def census(dtype, P, rung_seed, K=11, off_row=5):
    """The test's data (tests/test_generic_keys.py::test_reference_kernel_tile_rungs):
    vector path, scalar path (row ``off_row`` off 16-B alignment) and the
    reference's CPU arithmetic."""
    from oracle.reference_loop import ReferenceSerialAggregator

    dev = torch.device("cuda:0")
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(17 + rung_seed)
    X = [(torch.randn(P, generator=g, dtype=torch.float32) * 0.5).to(dt) for _ in range(K)]
    w = [int(v) for v in torch.randint(1, 600, (K,), generator=g)]
    w[2] = 0.37
    ref = ReferenceSerialAggregator()
    for k in range(K):
        ref.add("p", X[k], w[k])
    want = ref.get_sum("p")
    rows = [x.to(dev) for x in X]
    vec = torch.empty(P, dtype=dt, device=dev)
    ops.reduce_rows_ref(rows, w, vec)
    big = torch.empty(P + 1, dtype=dt, device=dev)
    big[1:].copy_(X[off_row])
    srows = list(rows)
    srows[off_row] = big[1:]
    sca = torch.empty(P, dtype=dt, device=dev)
    ops.reduce_rows_ref(srows, w, sca)
    vec, sca = vec.cpu(), sca.cpu()
    out = dict(dtype=dtype, P=P, K=K, off_row=off_row)
    for name, got in (("vec", vec), ("sca", sca)):
        bad = (got.double() != want.double()) & ~(got.isnan() & want.isnan())
        n = int(bad.sum())
        out[name + "_mismatches"] = n
        if n:
            idx = bad.nonzero().flatten()[:6].tolist()
            out[name + "_first"] = [dict(i=i, got=float(got[i]), want=float(want[i]),
                                         xs=[float(x[i]) for x in X]) for i in idx]
    print(json.dumps(out), flush=True)


def small_f16():
    """tests/golden generic scenario f16_matrix_int_weights through the kernel in
    two calls of two rows (max_rows=2), vs the reference's CPU arithmetic."""
    from oracle import generic_cases as G
    from oracle.reference_loop import ReferenceSerialAggregator

    dev = torch.device("cuda:0")
    ws = [5, 9, 1, 60]
    xs = [G.S("f16", (7, 33), 150 + i).build().reshape(-1) for i in range(4)]
    ref = ReferenceSerialAggregator()
    wants = []
    for x, w in zip(xs, ws):
        ref.add("m", x, w)
        wants.append(ref.get_sum("m"))
    rows = [x.to(dev) for x in xs]
    P = xs[0].numel()
    for split in (1, 2, 4):
        acc = None
        for lo in range(0, 4, split):
            out = torch.empty(P, dtype=torch.float16, device=dev)
            ops.reduce_rows_ref(rows[lo:lo + split], ws[lo:lo + split], out, acc_in=acc)
            acc = out
            got = out.cpu()
            want = wants[lo + split - 1]
            bad = (got.view(torch.int16) != want.view(torch.int16)).nonzero().flatten().tolist()
            rec = dict(split=split, upto=lo + split, mismatches=len(bad))
            if bad:
                rec["first"] = [dict(i=i, got=float(got[i]), want=float(want[i]),
                                     xs=[float(x[i]) for x in xs]) for i in bad[:6]]
            print(json.dumps(rec), flush=True)


def main():
    small_f16()
    census("float16", 8_400_005, 0)
    census("float16", 8_400_005, 0, off_row=0)
    census("float16", 4_200_007, 1)
    census("float16", 999, 2)
    census("bfloat16", 8_400_003, 0)
    census("float64", 3_200_001, 0)


if __name__ == "__main__":
    main()
