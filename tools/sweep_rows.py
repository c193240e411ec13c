"""Row-pointer (borrowed HBM-resident clients) reduce: buffer-descriptor vs
flat loads across unroll / float4-slots-per-lane, K separate client tensors,
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
Also times the fused last-drain + FedAvg step (fedagg_reduce_step_rows_f32)
with buffer and flat loads.  Every variant is checked bit for bit against the
first one.

python tools/sweep_rows.py [--K 1000] [--P 25000000] [--rounds 3]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

SHAPES = ((2, 4), (4, 2), (4, 4), (8, 1), (8, 2), (8, 4), (16, 1), (16, 2), (4, 1))
NARROW = (("narrow1", 8), ("narrow1", 16), ("narrow2", 8), ("narrow2", 16), ("narrow4", 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    K, P = a.K, a.P
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    rows = []
    for _ in range(K):  # K separate allocations, like borrowed client tensors
        rows.append(torch.empty(P, device=dev).normal_(0, 1, generator=g))
    table = ops.row_table(rows, dev)
    w32 = torch.randint(50, 601, (K,), device=dev).float()
    out = torch.empty(P, device=dev)
    ref = torch.empty(P, device=dev)
    ops.reduce_rows(rows, w32, ref, W=1.0,
                    flags=ops.tuning_flags(unroll=4, vpt=2, flat=True, mapping="wide"),
                    table=table)
    cloud0 = torch.empty(P, device=dev).normal_(0, 0.05, generator=g)
    cloud = cloud0.clone()
    cloud_ref = None

    variants = [dict(kind="reduce", unroll=u, vpt=v, flat=f, mapping="wide")
                for f in (False, True) for u, v in SHAPES]
    variants += [dict(kind="reduce", unroll=u, mapping=m, flat=False) for m, u in NARROW]
    variants += [dict(kind="step", flat=f, mapping="wide") for f in (False, True)]
    variants += [dict(kind="step", flat=False, mapping="auto")]
    times = {i: [] for i in range(len(variants))}
    for r in range(a.rounds):
        for i, var in enumerate(variants):
            if var["kind"] == "reduce":
                fl = ops.tuning_flags(unroll=var["unroll"], vpt=var.get("vpt", 0), nt=True,
                                      flat=var["flat"], mapping=var["mapping"])

                def run():
                    ops.reduce_rows(rows, w32, out, W=1.0, flags=fl, table=table)
            else:
                step = ops.ServerStep("fedavg", cloud, lr=1.0)

                def run():
                    cloud.copy_(cloud0)  # timed separately below; same in every variant
                    ops.reduce_rows_step(rows, w32, step, W=1.0, table=table, flat=var["flat"],
                                         mapping=var["mapping"])

            run()
            torch.cuda.synchronize()
            if r == 0:
                if var["kind"] == "reduce":
                    assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), var
                elif cloud_ref is None:
                    cloud_ref = cloud.clone()
                else:
                    assert torch.equal(cloud.view(torch.int32), cloud_ref.view(torch.int32)), var
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
    # the step variants include one P-sized copy (8P bytes) per iteration
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        cloud.copy_(cloud0)
    e1.record()
    torch.cuda.synchronize()
    copy_ms = e0.elapsed_time(e1) / a.iters
    res = []
    for i, var in enumerate(variants):
        ms = float(np.median(times[i]))
        if var["kind"] == "step":
            ms -= copy_ms
            alg = 4.0 * K * P + 4.0 * K + 12.0 * P
        else:
            alg = 4.0 * K * P + 4.0 * K + 4.0 * P
        res.append(dict(var, K=K, P=P, ms_median=ms, ms_min=float(np.min(times[i])),
                        GBps_alg=alg / ms / 1e6, GBps_client=4.0 * K * P / ms / 1e6))
    res.sort(key=lambda d: d["ms_median"])
    for d in res:
        print(json.dumps(d), flush=True)
    print(json.dumps({"copy_ms_subtracted_from_step": copy_ms}), flush=True)


if __name__ == "__main__":
    main()
