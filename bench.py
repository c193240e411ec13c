"""Benchmark: client-update bytes/s reduced (device-resident), K clients x P params.

One step = one FedAvg server round on the MI355X, device-resident: the
weighted exact-mode reduction of K client rows, the pop divide and the FedAvg
server SGD step (pseudo-gradient stored as cloud.grad) in ONE pass over the
slab (fedagg_reduce_step_blocked_f32) -- what SerialAggregator.add x K +
FedAvg.optimize does in this package.  Reference: SerialAggregator.add / pop
(fedsim/utils/aggregators.py:23-122) + FedAvg.optimize
(fedsim/distributed/centralized/training/fedavg.py:193-208), with the client
vectors already packed in HBM.  --step split times the two-launch variant
(reduce + divide, then the epilogue kernel).

Multi-GPU (launched by torch.distributed.run): parameter-sharded weak scaling,
SURVEY §8e — rank g owns a contiguous P-column shard of an N*P-parameter model
and reduces all K clients over it; no data-path collective (a barrier and a
max-over-ranks of the elapsed time only).  value = 4*K*P*N / max_time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fedsim_amd import ops  # noqa: E402

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "client-update bytes/s reduced (device-resident), K clients × P params"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--K", type=int, default=1000, help="clients per round")
    ap.add_argument("--P", type=int, default=25_000_000, help="params per GPU shard")
    ap.add_argument("--layout", default="blocked", choices=["blocked", "strided"],
                    help="HBM slab layout (blocked: column blocks of C floats, rows "
                         "contiguous inside a block; strided: row-major [K, ldx])")
    ap.add_argument("--C", type=int, default=4096, choices=[1024, 2048, 4096])
    ap.add_argument("--unroll", type=int, default=4, choices=[0, 2, 4, 8, 16])
    ap.add_argument("--vpt", type=int, default=2, choices=[0, 1, 2, 4],
                    help="float4 slots per lane (strided layout only)")
    ap.add_argument("--nt", type=int, default=1)
    ap.add_argument("--step", default="fused", choices=["fused", "split"],
                    help="fused: server step inside the reduce pass (the product path); "
                         "split: reduce + divide, then a separate epilogue launch")
    ap.add_argument("--mapping", default="auto", choices=["auto", "wide", "narrow1", "narrow2"],
                    help="column mapping of the reduce kernel (include/fedagg.h "
                         "FEDAGG_MAP_*); auto = the library's choice for P")
    ap.add_argument("--no-epilogue", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    pg = None
    # any torch.distributed.run launch (even --nproc-per-node 1) takes the
    # process-group path, so the N=1 rehearsal exercises the same barrier /
    # max-over-ranks code the N>1 runs use
    if world > 1 or ("MASTER_ADDR" in os.environ and "RANK" in os.environ):
        import torch.distributed as dist

        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        pg = dist
    return world, rank, local, pg


def make_inputs(K, P, rank, dev, layout, C):
    """x_k = base + eps_k, base ~ N(0, 0.05) (seed 7), eps_k ~ N(0, 1e-3)
    (Philox, seed 20261015 + row block); FedAvg weights w_k ~ U{50..600}
    (numpy seed 11).

    strided: row-major [K, ldx] fp32 slab, 256-B aligned rows.
    blocked: [ceil(P/C), K, C] — column block b holds rows 0..K-1 of columns
             [bC, bC+C) contiguously (include/fedagg.h), the layout the
             aggregator packs client vectors into."""
    g = torch.Generator(device=dev)
    g.manual_seed(7 + 1_000_003 * rank)
    base = torch.empty(P, dtype=torch.float32, device=dev).normal_(0.0, 0.05, generator=g)
    blk = 64
    if layout == "strided":
        ldx = (P + 63) // 64 * 64
        X = torch.empty((K, ldx), dtype=torch.float32, device=dev)
    else:
        X = torch.zeros(ops.blocked_shape(K, P, C), dtype=torch.float32, device=dev)
        tmp = torch.empty((blk, P), dtype=torch.float32, device=dev)
        full = P // C
    for k0 in range(0, K, blk):
        k1 = min(K, k0 + blk)
        g.manual_seed(20261015 + k0 + 1_000_003 * rank)
        if layout == "strided":
            X[k0:k1, :P].normal_(0.0, 1e-3, generator=g).add_(base)
        else:
            t = tmp[: k1 - k0].normal_(0.0, 1e-3, generator=g).add_(base)
            X[:full, k0:k1, :].copy_(t[:, : full * C].view(k1 - k0, full, C).transpose(0, 1))
            if P % C:
                X[full, k0:k1, : P % C].copy_(t[:, full * C:])
    del base
    weights = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    return X, weights


def load_pmc(path, K, P, kernel, layout, step):
    """HBM bytes per launch from the committed PMC summary
    (tools/pmc_traffic.py), when it was measured on this exact kernel and
    workload; else None."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("K") == K and d.get("P") == P and d.get("kernel") == kernel and \
            d.get("layout", "strided") == layout and d.get("step", "split") == step:
        return d.get("hbm_bytes_per_launch")
    return None


def cpu_baseline(P, budget_s):
    """The reference's per-client loop restated on torch CPU (oracle leg),
    timed on a bounded sample of the same workload: distinct client tensors of
    the headline P, as many clients as fit ~budget_s of host time."""
    from oracle.reference_loop import aggregate_round

    threads = torch.get_num_threads()
    rng = np.random.default_rng(11)
    pool_n = 8
    pool = [torch.randn(P) for _ in range(pool_n)]
    weights = [int(v) for v in rng.integers(50, 601, size=4096)]
    t0 = time.perf_counter()
    aggregate_round(pool[:2], weights[:2])
    per_client = (time.perf_counter() - t0) / 2
    n = int(max(4, min(2000, budget_s / max(per_client, 1e-6))))
    rows = [pool[k % pool_n] for k in range(n)]
    t0 = time.perf_counter()
    aggregate_round(rows, weights[:n])
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        cpu = platform.processor()
    return dict(
        value=4.0 * n * P / dt / 1e9,
        unit="GB/s",
        cores=threads,
        kind="port",
        sample=(f"oracle/reference_loop.aggregate_round (torch CPU clone + mul + add per client, "
                f"then divide) over {n} clients x P={P} fp32 (pool of {pool_n} distinct host "
                f"tensors), {dt:.2f} s on {threads} threads of {cpu}"),
    )


class _StdoutToStderr(object):
    """Route file descriptor 1 to stderr until the result line is printed,
    so that banners written by native libraries (RCCL prints its version
    block to stdout at communicator init) cannot join the ONE JSON line the
    driver reads from stdout."""

    def __init__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def restore(self):
        if self.saved is None:
            return
        sys.stdout.flush()
        try:  # C stdio buffers written while fd 1 was stderr go there too
            import ctypes

            ctypes.CDLL(None).fflush(None)
        except (OSError, AttributeError):
            pass
        os.dup2(self.saved, 1)
        os.close(self.saved)
        self.saved = None


def main():
    quiet = _StdoutToStderr()
    try:
        _main(quiet)
    finally:
        quiet.restore()


def _main(quiet):
    a = parse()
    world, rank, local, dist = dist_setup()
    dev = torch.device("cuda", local)
    K, P = a.K, a.P
    flags = ops.tuning_flags(unroll=a.unroll, vpt=a.vpt if a.layout == "strided" else 0,
                             nt=bool(a.nt), mapping=a.mapping)
    fused = a.step == "fused" and a.layout == "blocked" and not a.no_epilogue
    step_mode = "fused" if fused else "split"
    X, weights = make_inputs(K, P, rank, dev, a.layout, a.C)
    W = sum(weights)
    w32 = torch.tensor([ops.fl32(v) for v in weights], dtype=torch.float32, device=dev)
    avg = torch.empty(P, dtype=torch.float32, device=dev)
    cloud = torch.zeros(P, dtype=torch.float32, device=dev)
    grad = torch.empty(P, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    # FedAvg.optimize's server step (default SGD lr 1.0, fed_learn.py:129),
    # cloud.grad = pseudo-gradient as torch leaves it
    sstep = ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad)

    def reduce():
        if fused:
            ops.reduce_blocked_step(X, w32, sstep, W=W, mapping=a.mapping)
        elif a.layout == "strided":
            ops.reduce_slab(X[:, :P], w32, avg, W=W, P=P, flags=flags)
        else:
            ops.reduce_blocked(X, w32, avg, W=W, flags=flags)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        reduce()
        if ev is not None:
            ev[1].record(stream)
        if not a.no_epilogue and not fused:
            ops.fedavg_sgd(avg, cloud, 1.0, grad_out=grad)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    total_bytes = 4.0 * K * P * world
    value = total_bytes * a.steps / elapsed / 1e9
    # client rows + weights, plus per column: fused = cloud read + cloud write +
    # grad write; split (reduce kernel alone) = the average's write
    alg_bytes_launch = 4.0 * K * P + 4.0 * K + (12.0 * P if fused else 4.0 * P)
    achieved = alg_bytes_launch / (kern_ms * 1e-3) / 1e9
    # the kernel the library launched: the fused step path takes only the
    # mapping bits, the plain reduce all of `flags`
    mapping, unroll = ops.column_mapping(
        P, ops.tuning_flags(mapping=a.mapping) if fused else flags, B=K)
    kernel = ("k_reduce_vec" if mapping == "wide" else
              f"k_reduce_narrow<U={unroll}, VW={mapping[-1]}>")
    traffic = load_pmc(a.pmc_json, K, P, kernel,
                       a.layout if a.layout == "strided" else f"blocked{a.C}", step_mode)
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (x_k = base + eps_k on device, FedAvg int weights U{50..600})",
        "config": {
            "workload": ("FedAvg server round, device-resident: exact weighted reduce + divide "
                         "+ SGD server step in one pass" if fused else
                         "FedAvg server round, device-resident: exact weighted reduce + divide, "
                         "then the SGD epilogue kernel"),
            "step": step_mode,
            "clients_K": K,
            "params_per_gpu_P": P,
            "params_total": P * world,
            "parallelism": f"param-shard{world}" if world > 1 else "single",
            "mode": "exact (bitwise vs reference CPU)",
            "layout": a.layout if a.layout == "strided" else f"blocked C={a.C}",
            "mapping": mapping if mapping == "wide" else f"{mapping} (U={unroll})",
            "flags": flags,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "%s (%s)" % (kernel,
                "fedagg_reduce_step_blocked_f32, EpiStep<FEDAVG>" if fused else
                "fedagg_reduce_blocked_f32" if a.layout == "blocked" else "fedagg_reduce_f32"),
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBPS, 4),
            "traffic": traffic,
            "launch_ms": round(kern_ms, 4),
            "alg_bytes_per_launch": alg_bytes_launch,
        },
    }
    del X
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(P, a.cpu_baseline_seconds)
    if rank == 0:
        quiet.restore()
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
