"""Per-config measurements of the aggregation path (BASELINE.json configs 1-5),
device-resident, exact mode unless noted.  Complements bench.py (the headline
K=1000 x P=25M line) with the sizes the reference's own configs use.

  cfg1  FedAvg, SimpleMLP P=199,210, K=5            (latency: one round)
  cfg2  FedAvg, SimpleCNN2 P=1,085,668, K=10 / 1000
  cfg3  AdaBest beta=0.6, SimpleCNN2 P=1,085,668, K=10 / 1000 (w=1, AdaBest epilogue)
  cfg4  FedAvg synthetic, param-sharded: per-GPU shard K=10,000 x P=25M/8
  cfg5  FedAvg synthetic, client-sharded: per-GPU K=12,500 x P=125M streamed from a
        resident 200-row pool (re-read cyclically), + RCCL all-reduce(4P) when N>1

One process per GPU under torch.distributed.run for N>1 (cfg4/cfg5 only).
python tools/bench_configs.py [--only cfg2,cfg5] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd import ops  # noqa: E402

def blocked_random(K, P, dev, seed):
    C = ops.choose_block_cols(P)
    Xb = torch.empty(ops.blocked_shape(K, P, C), device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    for b0 in range(0, Xb.shape[0], 256):
        Xb[b0:b0 + 256].normal_(0.0, 0.05, generator=g)
    return Xb


def timed(fn, steps, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def gpu_time(fn, steps):
    """Median time of one isolated call between two HIP events on the current
    stream, synchronized each time: includes the launch latency of an idle
    GPU, which back-to-back calls (the wall-clock rate) overlap.  Kernel-only
    times come from rocprofv3."""
    ms = []
    for _ in range(steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms)) * 1e-3


def round_exact(Xb, w32, W, P, epilogue=None, pool_passes=1, K_pool=None, fused=False):
    """One round: pool_passes reduce passes (+ divide in the last), then the
    server step.  fused=True runs the step inside the last pass
    (fedagg_reduce_step_blocked_f32, what <Algo>.optimize does), writing the
    pseudo-gradient too as the product path does."""
    dev = Xb.device
    avg = torch.empty(P, device=dev)
    cloud = torch.zeros(P, device=dev)
    prev = torch.zeros(P, device=dev)
    grad = torch.empty(P, device=dev)
    step = None
    if fused and epilogue:
        step = ops.ServerStep(epilogue, cloud, lr=1.0, coef=0.6 if epilogue == "adabest" else 0.0,
                              aux=prev if epilogue == "adabest" else None, grad_out=grad)

    def fn():
        for i in range(pool_passes):
            last = i == pool_passes - 1
            if last and step is not None:
                ops.reduce_blocked_step(Xb, w32, step, B=K_pool,
                                        acc_in=None if i == 0 else avg, W=W)
                continue
            ops.reduce_blocked(Xb, w32, avg, B=K_pool, acc_in=None if i == 0 else avg,
                               W=W if last else None, flags=ops.default_flags(Xb.shape[2]))
        if step is not None:
            return avg
        if epilogue == "fedavg":
            ops.fedavg_sgd(avg, cloud, 1.0)
        elif epilogue == "adabest":
            ops.adabest_sgd(avg, cloud, prev, 0.6, 1.0)
        return avg

    return fn, avg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg1,cfg2,cfg3,cfg4,cfg5")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cfg5-pool", type=int, default=200,
                    help="resident client rows config 5 streams from (200 x 500 MB = 100 GB; "
                         "each extra pass costs 8P bytes of accumulator traffic)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
    rng = np.random.default_rng(11)
    out = {}
    only = set(a.only.replace("+", ",").split(","))

    def report(name, K, P, t, extra=None):
        bytes_ = 4.0 * K * P * world
        r = dict(K_per_gpu=K, P_per_gpu=P, n_gpus=world, ms=t * 1e3, GBps=bytes_ / t / 1e9,
                 C=ops.choose_block_cols(P))
        if extra:
            r.update(extra)
        out[name] = r
        if rank == 0:
            print(json.dumps({name: r}), flush=True)

    for name, K, P, epi in (("cfg1", 5, 199_210, "fedavg"), ("cfg2_K10", 10, 1_085_668, "fedavg"),
                            ("cfg2_K1000", 1000, 1_085_668, "fedavg"),
                            ("cfg3_K10", 10, 1_085_668, "adabest"),
                            ("cfg3_K1000", 1000, 1_085_668, "adabest")):
        if name.split("_")[0] not in only or world > 1:
            continue
        Xb = blocked_random(K, P, dev, 1)
        ws = [1] * K if epi == "adabest" else [int(v) for v in rng.integers(50, 601, size=K)]
        w32 = torch.tensor([ops.fl32(v) for v in ws], device=dev)
        for fused in (True, False):
            fn, _ = round_exact(Xb, w32, sum(ws), P, epilogue=epi, fused=fused)
            t = timed(fn, max(a.steps, 20))
            gt = gpu_time(fn, max(a.steps, 20))
            report(name + ("" if fused else "_split"), K, P, t,
                   dict(epilogue=epi, step="fused into the last reduce" if fused
                        else "separate epilogue launch", isolated_call_ms=gt * 1e3))
        del Xb

    if "cfg4" in only:
        K, P = 10_000, 25_000_000 // 8
        Xb = blocked_random(K, P, dev, 2 + rank)
        ws = [int(v) for v in rng.integers(50, 601, size=K)]
        w32 = torch.tensor([ops.fl32(v) for v in ws], device=dev)
        fn, _ = round_exact(Xb, w32, sum(ws), P, epilogue="fedavg", fused=True)
        if dist is not None:
            dist.barrier()
        report("cfg4_param_shard", K, P, timed(fn, a.steps),
               dict(note="per-GPU shard of a 10,000 x 25M round (x8 = full model)"))
        del Xb
        torch.cuda.empty_cache()

    if "cfg5" in only:
        K, P, pool = 12_500, 125_000_000, a.cfg5_pool
        counts = [min(pool, K - k0) for k0 in range(0, K, pool)]  # the last pass may be short
        Xb = blocked_random(pool, P, dev, 3 + rank)
        ws = [int(v) for v in rng.integers(50, 601, size=pool)]
        w32 = torch.tensor([ops.fl32(v) for v in ws], device=dev)
        W_total = sum(sum(ws[:n]) for n in counts) * world
        acc = torch.empty(P, device=dev)

        def fn():
            for i, n in enumerate(counts):
                ops.reduce_blocked(Xb, w32, acc, B=n, acc_in=None if i == 0 else acc,
                                   flags=ops.default_flags(Xb.shape[2]))
            if dist is not None:
                dist.all_reduce(acc)
            ops.finalize(acc, W_total, out=acc)

        if dist is not None:
            dist.barrier()
        report("cfg5_client_shard_allreduce", K, P, timed(fn, max(1, a.steps // 2), warmup=1),
               dict(pool_rows=pool, passes=len(counts),
                    note=f"K_per_gpu streamed from a resident {pool * P * 4 / 1e9:.0f} GB pool; "
                         "RCCL all-reduce of 4P bytes when N>1"))
        del Xb

    if rank == 0:
        print(json.dumps({"all": out}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
