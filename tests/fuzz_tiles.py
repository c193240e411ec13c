"""Time-boxed random fuzzing of the row-table reductions (GPU): the generic
keys' kernel (fedagg_reduce_rows_ref, bf16 / fp16 / fp64) against the
reference's own CPU arithmetic (oracle/reference_loop, ATen), and
fedagg_reduce_rows_f32 (wide tiles or narrow kernels by size) against the
narrow kernels with the mapping forced and against numpy float32 on sampled
columns.  Random P (log-uniform, 1 .. 9 M), K, weights (integers, tie-prone
decimals, negatives, zero), values (normal at several scales, with +-0,
+-inf, NaN, subnormals and huge values mixed in), a row off 16-B alignment,
and a running sum continued through acc_in; and whole fp32 drop-in
sessions (agg: HBM / host rows, borrowed or not, ring drains, a get
mid-stream) against the reference's CPU SerialAggregator.  NaN positions are compared as
NaN (their bits are not pinned by the reference).  Prints one JSON line per
100 cases and a summary; exit 1 on the first mismatch, with the case.

python tests/fuzz_tiles.py [--seconds 300] [--seed 1] [--min-p 1]

(a GPU script kept with the tests, not collected by pytest: the oracle is its
checker)
"""
import argparse
import json
import math
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402
from oracle.reference_loop import ReferenceSerialAggregator  # noqa: E402

MAP_VW2 = 3 << 18
SPECIALS = [0.0, -0.0, math.inf, -math.inf, math.nan, 1e-42, 3e-39, 6.5e4, 3e38]
MIN_P = 1


def draw_p(rng, hi):
    lo = min(MIN_P, hi)
    return int(math.exp(rng.uniform(math.log(lo), math.log(hi))))


def values(rng, P, K, dt, special):
    scale = rng.choice([1e-3, 0.5, 30.0, 6e4 if dt != torch.float64 else 1e200])
    g = torch.Generator().manual_seed(rng.randrange(1 << 30))
    X = torch.randn(K, P, generator=g, dtype=torch.float64) * scale
    if special:
        n = max(1, K * P // rng.choice([20, 200, 5000]))
        idx = torch.randint(0, K * P, (n,), generator=g)
        vals = torch.tensor(SPECIALS, dtype=torch.float64)
        X.view(-1)[idx] = vals[torch.randint(0, len(SPECIALS), (n,), generator=g)]
    return X.to(dt)


def weights(rng, K):
    pool = [lambda: rng.randint(1, 600), lambda: rng.randint(-50, 50), lambda: 0,
            lambda: rng.choice([0.37, 0.1, 1 / 3, 0.7, 2.75, 1e-3]),
            lambda: rng.uniform(-4, 4)]
    return [rng.choice(pool)() for _ in range(K)]


def same(got, want, ib):
    ng, nw = torch.isnan(got), torch.isnan(want)
    return bool(torch.equal(ng, nw) and torch.equal(got[~ng].view(ib), want[~nw].view(ib)))


def generic_case(rng, dev):
    dt = rng.choice([torch.bfloat16, torch.float16, torch.float64])
    P = draw_p(rng, 9_000_000 if dt != torch.float64 else 3_600_000)
    K = rng.randint(1, 12)
    special = rng.random() < 0.3
    X = values(rng, P, K, dt, special)
    w = weights(rng, K)
    ref = ReferenceSerialAggregator()
    for k in range(K):
        ref.add("p", X[k], w[k])
    want = ref.get_sum("p")
    rows = [X[k].to(dev) for k in range(K)]
    off = rng.randrange(K) if rng.random() < 0.3 else None
    if off is not None:
        big = torch.empty(P + 1, dtype=dt, device=dev)
        big[1:].copy_(rows[off])
        rows[off] = big[1:]
    out = torch.empty(P, dtype=dt, device=dev)
    split = rng.randint(0, K)
    if 0 < split < K:
        head = torch.empty(P, dtype=dt, device=dev)
        ops.reduce_rows_ref(rows[:split], w[:split], head)
        ops.reduce_rows_ref(rows[split:], w[split:], out, acc_in=head)
    else:
        ops.reduce_rows_ref(rows, w, out)
    ib = torch.int64 if dt == torch.float64 else torch.int16
    ok = same(out.cpu(), want, ib)
    return ok, dict(kind="generic", dtype=str(dt), P=P, K=K, w=w, special=special, off=off,
                    split=split)


def f32_case(rng, dev):
    P = draw_p(rng, 9_000_000)
    K = rng.randint(1, 16)
    special = rng.random() < 0.2
    X = values(rng, P, K, torch.float32, special)
    wl = weights(rng, K)
    w32 = torch.tensor([ops.fl32(x) for x in wl], dtype=torch.float32, device=dev)
    rows = [X[k].to(dev) for k in range(K)]
    W = sum(wl) if rng.random() < 0.5 and sum(wl) != 0 else None
    split = rng.randint(0, K)
    outs = []
    for flags in (0, MAP_VW2):
        out = torch.empty(P, device=dev)
        if 0 < split < K:
            acc = torch.empty(P, device=dev)
            ops.reduce_rows(rows[:split], w32[:split], acc, flags=flags)
            ops.reduce_rows(rows[split:], w32[split:], acc, acc_in=acc, W=W, flags=flags)
            out = acc
        else:
            ops.reduce_rows(rows, w32, out, W=W, flags=flags)
        outs.append(out)
    ok = same(outs[0].cpu(), outs[1].cpu(), torch.int32)
    # numpy float32 on sampled columns: the reference's per-column arithmetic
    cols = np.unique(np.random.default_rng(rng.randrange(1 << 30)).integers(0, P, min(P, 512)))
    Xs = X[:, cols].numpy()
    with np.errstate(all="ignore"):
        s = np.zeros(len(cols), np.float32)
        for k in range(K):
            s = np.float32(s + np.float32(Xs[k] * np.float32(wl[k])))
        if W is not None:
            s = np.float32(s / np.float32(W))
    ok = ok and same(outs[0][torch.from_numpy(cols).to(dev)].cpu(), torch.from_numpy(s), torch.int32)
    return ok, dict(kind="f32", P=P, K=K, w=wl, special=special, W=W, split=split)


def agg_case(rng, dev):
    """A whole drop-in session on fp32 client vectors: HBM (borrowed or
    snapshotted) or host rows, ring drains at a random max_rows, a get
    mid-stream, then pop -- against the reference's CPU SerialAggregator."""
    from fedsim_amd.utils import SerialAggregator

    P = draw_p(rng, 4_000_000)
    K = rng.randint(1, 24)
    special = rng.random() < 0.2
    X = values(rng, P, K, torch.float32, special)
    w = [x if rng.random() < 0.7 else float(x) for x in weights(rng, K)]
    borrow = rng.random() < 0.5
    agg = SerialAggregator(max_rows=rng.randint(1, 30), borrow=borrow)
    ref = ReferenceSerialAggregator()
    where = [rng.choice(["hbm", "hbm", "host"]) for _ in range(K)]
    mid = rng.randrange(K)
    ok = True
    for k in range(K):
        v = X[k].to(dev) if where[k] == "hbm" else X[k].clone()
        agg.add("p", v, w[k])
        ref.add("p", X[k], w[k])
        if k == mid:
            g, e = agg.get("p"), ref.get("p")
            ok = ok and same(g.cpu() if isinstance(g, torch.Tensor) else g, e, torch.int32)
    got, want = agg.pop("p"), ref.pop("p")
    ok = ok and same(got.cpu(), want, torch.int32)
    return ok, dict(kind="agg", P=P, K=K, w=w, special=special, borrow=borrow, where=where,
                    mid=mid)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--min-p", type=int, default=1, help="smallest P drawn (the tiles: 1000000)")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    global MIN_P
    MIN_P = a.min_p
    dev = torch.device("cuda:0")
    t0, n, counts = time.time(), 0, {"generic": 0, "f32": 0, "agg": 0}
    while time.time() - t0 < a.seconds:
        kind = rng.choice(["generic", "f32", "agg"])
        ok, case = {"generic": generic_case, "f32": f32_case, "agg": agg_case}[kind](rng, dev)
        n += 1
        counts[kind] += 1
        if not ok:
            print(json.dumps(dict(mismatch=case)), flush=True)
            sys.exit(1)
        if n % 100 == 0:
            print(json.dumps(dict(cases=n, seconds=round(time.time() - t0, 1), **counts)), flush=True)
    print(json.dumps(dict(done=True, cases=n, seconds=round(time.time() - t0, 1), **counts)),
          flush=True)


if __name__ == "__main__":
    main()
