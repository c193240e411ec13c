"""Benchmark: client-update bytes/s reduced (device-resident), K clients x P params.

One step = one FedAvg server round on the MI355X, device-resident: the exact
weighted reduction of K client rows, the pop divide and the FedAvg server SGD
step (pseudo-gradient stored as cloud.grad) -- what SerialAggregator.add x K +
FedAvg.optimize does in this package.  Reference: SerialAggregator.add / pop
(fedsim/utils/aggregators.py:23-122) + FedAvg.optimize
(fedsim/distributed/centralized/training/fedavg.py:193-208), with the client
vectors already packed in HBM.

Modes (``--mode``), one process per GPU, SURVEY §8e:

* ``param`` (default; the headline, BASELINE configs[1]'s K=1000 x P=25 M per
  GPU): weak scaling.  Rank g owns a contiguous 25 M-column shard of an
  N*25 M-parameter model and runs the round over all K clients on it: ONE
  launch of fedagg_reduce_step_blocked_f32 (reduce + divide + server step in
  one pass).  No data-path collective.  value = 4*K*P*N / max-over-ranks time.
* ``strong`` (config 4): FedAvg 10 000 clients x 25 M params in total,
  parameter-sharded over N GPUs (64-aligned column shards, no collective).  A
  shard that does not fit HBM (N <= 2) streams from a resident pool of
  distinct client rows, chained through the accumulator (declared in the line).
* ``allreduce`` (config 5): client-sharded, 12 500 clients x 125 M params per
  GPU (x8 = 100 000), streamed from a resident 200-row pool, then ONE RCCL
  all-reduce(sum) of the 4P-byte partial over xGMI, the divide by fl32(W) and
  the server step.  The all-reduce's share of the round is reported
  separately.  Reordered sum: normwise parity.

Launch: ``python bench.py --gpus N`` spawns N rank processes itself (before
anything touches a GPU) when it is not already running under
torch.distributed.run; either way rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "client-update bytes/s reduced (device-resident), K clients × P params"
# per-mode workload defaults: (K, P, K means) -- BASELINE.json configs 1, 4, 5
MODE_DEFAULTS = {
    "param": (1000, 25_000_000, "clients per round; P per GPU shard"),
    "strong": (10_000, 25_000_000, "clients per round; P = whole model, sharded over N"),
    "allreduce": (12_500, 125_000_000, "clients per GPU (x N in total); P = whole model"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed rounds (default 20; 5 for strong, 3 for allreduce)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed rounds (default 3; 1 for strong / allreduce)")
    ap.add_argument("--mode", default="param", choices=sorted(MODE_DEFAULTS))
    ap.add_argument("--K", type=int, default=None, help="clients (see --mode)")
    ap.add_argument("--P", type=int, default=None, help="params (see --mode)")
    ap.add_argument("--pool-rows", type=int, default=None,
                    help="resident client rows the streamed modes re-read (allreduce: 200; "
                         "strong: as many as fit)")
    ap.add_argument("--layout", default="blocked", choices=["blocked", "strided"],
                    help="param mode's HBM slab layout (blocked: column blocks of C floats, "
                         "rows contiguous inside a block; strided: row-major [K, ldx])")
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
    ap.add_argument("--no-side-legs", action="store_true",
                    help="skip the N=1 side legs after the headline (h2d_inclusive: the "
                         "host-to-host round; configs: BASELINE configs 2 / 3)")
    ap.add_argument("--no-selftest", action="store_true",
                    help="skip the multi-GPU self-test that precedes the timed region")
    ap.add_argument("--selftest-fault-rank", type=int, default=None,
                    help="TEST ONLY: flip one result bit on this rank in the self-test")
    ap.add_argument("--selftest-fault-devices", action="store_true",
                    help="TEST ONLY: fail rank 0's devices_* check in the self-test")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--master-port", type=int, default=0,
                    help="rendezvous port of the self-spawned ranks (0: pick a free one)")
    ap.add_argument("--one-gpu-rehearsal", action="store_true",
                    help="TEST ONLY: every rank on cuda:0 over a gloo group, to rehearse "
                         "the N-rank launcher with the HIP kernels on a one-GPU box (ranks "
                         "share the GPU: the value is not a scaling number)")
    ap.add_argument("--rehearsal-stub", default=None, metavar="MODULE:FN",
                    help="TEST ONLY: run the launcher and the collectives on CPU over gloo, "
                         "with the per-rank reduction done by MODULE:FN (no GPU, no HIP "
                         "kernel; the line is marked as a rehearsal and carries no roofline)")
    a = ap.parse_args(argv)
    K, P, _ = MODE_DEFAULTS[a.mode]
    a.K = K if a.K is None else a.K
    a.P = P if a.P is None else a.P
    heavy = a.mode != "param"
    a.steps = (3 if a.mode == "allreduce" else 5 if heavy else 20) if a.steps is None else a.steps
    a.warmup = (1 if heavy else 3) if a.warmup is None else a.warmup
    return a


# --------------------------------------------------------------------------
# launcher: N rank processes from a parent that never touches the GPU
# --------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a, argv):
    """Start ranks 0..N-1 of this script (one per GPU) as child processes with
    the torch.distributed.run environment, relay rank 0's result line, and
    return the worst exit code.  The parent imports neither torch's HIP runtime
    nor libfedagg, so nothing is initialised on a GPU before the children
    start; a rank that fails ends the others."""
    n = a.gpus
    port = a.master_port or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FEDSIM_BENCH_CHILD="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.abspath(__file__), *argv], env=env,
            stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    out = []
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        out = procs[0].stdout.read().splitlines()
    lines = [ln for ln in out if ln.startswith("{")]
    if rc == 0 and len(lines) != 1:
        sys.stderr.write("bench: rank 0 printed %d result lines\n" % len(lines))
        rc = 1
    for ln in out:
        if not ln.startswith("{"):
            sys.stderr.write(ln + "\n")
    if lines:
        print(lines[-1], flush=True)
    return rc


# --------------------------------------------------------------------------
# ranks
# --------------------------------------------------------------------------
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


class Rank(object):
    """This process's place in the job and its device plumbing."""

    def __init__(self, a):
        import torch

        self.torch = torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.rehearsal = a.rehearsal_stub is not None
        self.dist = None
        if self.rehearsal:
            mod, fn = a.rehearsal_stub.split(":")
            self.stub = getattr(importlib.import_module(mod), fn)
            self.dev = torch.device("cpu")
        else:
            self.local = 0 if a.one_gpu_rehearsal else self.local
            torch.cuda.set_device(self.local)
            self.dev = torch.device("cuda", self.local)
        # any torch.distributed.run launch (even --nproc-per-node 1) takes the
        # process-group path, so the N=1 rehearsal exercises the same barrier /
        # max-over-ranks code the N>1 runs use
        if self.world > 1 or ("MASTER_ADDR" in os.environ and "RANK" in os.environ):
            import torch.distributed as dist

            if self.rehearsal or a.one_gpu_rehearsal:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group(backend="nccl", device_id=self.dev)
            self.dist = dist

    def sync(self):
        if not self.rehearsal:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, *vals):
        if self.dist is None:
            return vals
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return tuple(float(v) for v in t.tolist())


class KernelClock(object):
    """Per-launch HIP events on the stream the library launches on (the
    current torch stream), so ``achieved`` is algorithmic bytes over kernel
    time, not over the round's wall clock."""

    def __init__(self, rk):
        self.rk = rk
        self.marks = []  # (bytes, ev0, ev1)
        self.on = False

    def run(self, nbytes, fn):
        if not self.on or self.rk.rehearsal:
            return fn()
        torch = self.rk.torch
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        self.marks.append((nbytes, e0, e1))
        return r

    def summary(self):
        """(algorithmic bytes per launch, mean launch ms)."""
        if not self.marks:
            return None, None
        ms = [e0.elapsed_time(e1) for _, e0, e1 in self.marks]
        nb = sum(b for b, _, _ in self.marks)
        return nb / len(self.marks), sum(ms) / len(ms)


def _weights(K, seed=11):
    import numpy as np

    return [int(v) for v in np.random.default_rng(seed).integers(50, 601, size=K)]


def make_inputs(rk, K, P, layout, C):
    """x_k = base + eps_k, base ~ N(0, 0.05) (seed 7), eps_k ~ N(0, 1e-3)
    (Philox, seed 20261015 + row block); FedAvg weights w_k ~ U{50..600}
    (numpy seed 11).

    strided: row-major [K, ldx] fp32 slab, 256-B aligned rows.
    blocked: [ceil(P/C), K, C] -- column block b holds rows 0..K-1 of columns
             [bC, bC+C) contiguously (include/fedagg.h), the layout the
             aggregator packs client vectors into."""
    from fedsim_amd import ops

    torch, dev, rank = rk.torch, rk.dev, rk.rank
    g = torch.Generator(device=dev)
    g.manual_seed(7 + 1_000_003 * rank)
    base = torch.empty(P, dtype=torch.float32, device=dev).normal_(0.0, 0.05, generator=g)
    blk = 64
    if layout == "strided" or rk.rehearsal:
        ldx = (P + 63) // 64 * 64
        X = torch.empty((K, ldx), dtype=torch.float32, device=dev)
    else:
        X = torch.zeros(ops.blocked_shape(K, P, C), dtype=torch.float32, device=dev)
        tmp = torch.empty((blk, P), dtype=torch.float32, device=dev)
        full = P // C
    for k0 in range(0, K, blk):
        k1 = min(K, k0 + blk)
        g.manual_seed(20261015 + k0 + 1_000_003 * rank)
        if layout == "strided" or rk.rehearsal:
            X[k0:k1, :P].normal_(0.0, 1e-3, generator=g).add_(base)
        else:
            t = tmp[: k1 - k0].normal_(0.0, 1e-3, generator=g).add_(base)
            X[:full, k0:k1, :].copy_(t[:, : full * C].view(k1 - k0, full, C).transpose(0, 1))
            if P % C:
                X[full, k0:k1, : P % C].copy_(t[:, full * C:])
    return X


def make_pool(rk, R, P, C, seed):
    """A resident pool of R distinct client rows, column-blocked [ceil(P/C),
    R, C], values N(0, 0.05) (Philox ``seed``): the streamed modes re-read it
    cyclically to stand for K >> R clients (footprint >> the 256 MB MALL)."""
    from fedsim_amd import ops

    torch = rk.torch
    g = torch.Generator(device=rk.dev).manual_seed(seed)
    if rk.rehearsal:
        return torch.empty((R, P)).normal_(0.0, 0.05, generator=g)
    Xb = torch.empty(ops.blocked_shape(R, P, C), dtype=torch.float32, device=rk.dev)
    for b0 in range(0, Xb.shape[0], 256):
        Xb[b0:b0 + 256].normal_(0.0, 0.05, generator=g)
    return Xb


def _md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def load_pmc(path, K, P, kernel, layout, step, lib_path):
    """HBM bytes per launch from the committed PMC summary
    (tools/pmc_traffic.py), with where it came from.  The bytes are reported
    only when the summary was measured on this exact kernel and workload AND
    on this build of libfedagg.so (md5 of the library this process loaded);
    otherwise traffic is None and the source says why.  Returns (traffic,
    source)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, dict(summary=os.path.relpath(path, REPO), reason=f"unreadable: {e}")
    src = dict(d.get("source") or {})
    src["summary"] = os.path.relpath(path, REPO)
    try:
        here = _md5(lib_path)
    except OSError:
        here = None
    src["lib_md5_loaded"] = here
    if not (d.get("K") == K and d.get("P") == P and d.get("kernel") == kernel and
            d.get("layout", "strided") == layout and d.get("step", "split") == step):
        src["reason"] = "the summary was measured on another kernel / workload"
        return None, src
    if src.get("lib_md5") is None or src.get("lib_md5") != here:
        src["reason"] = "the summary was measured on another build of libfedagg.so"
        return None, src
    src["reason"] = "same kernel, workload and build (PMC FETCH_SIZE + WRITE_SIZE passes)"
    return d.get("hbm_bytes_per_launch"), src


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Threads for the CPU baseline: every CPU this process may run on,
    capped by OMP_NUM_THREADS when the box sets it (the GPU pool sets it to
    the box's CPU share, 16 per GPU: nproc there shows the whole machine).
    Returns (threads, facts) -- facts go into the JSON line."""
    affinity = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity
    try:
        import psutil

        physical = psutil.cpu_count(logical=False)
    except Exception:  # noqa: BLE001 - optional fact
        physical = None
    return threads, dict(affinity_cpus=affinity, omp_num_threads=omp, physical_cores=physical,
                         logical_cpus=os.cpu_count(), cpu_model=_cpu_model())


def cpu_baseline(P, budget_s):
    """The reference's per-client loop restated on torch CPU (oracle leg),
    timed on a bounded sample of the same workload: distinct client tensors of
    the workload's P, as many clients as fit ~budget_s of host time."""
    import numpy as np
    import torch

    from oracle.reference_loop import aggregate_round

    threads, facts = cpu_threads()
    torch.set_num_threads(threads)
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
    return dict(
        value=4.0 * n * P / dt / 1e9,
        unit="GB/s",
        cores=threads,
        kind="port",
        threads_rule="torch.set_num_threads(min(len(os.sched_getaffinity(0)), OMP_NUM_THREADS))",
        **facts,
        sample=(f"oracle/reference_loop.aggregate_round (torch CPU clone + mul + add per client, "
                f"then divide) over {n} clients x P={P} fp32 (pool of {pool_n} distinct "
                f"{4 * P / 1e6:.0f} MB host tensors, far above L3), {dt:.2f} s on {threads} "
                f"threads of {facts['cpu_model']}"),
    )


# -- multi-GPU self-test (outside the timed region) -------------------------
SELFTEST_K, SELFTEST_P = 24, 20_011  # ~2 MB of client rows: seconds, not minutes


def _oracle_reduce(X, w32, out, acc_in, W):
    """Rehearsal stand-in for a rank's HIP reduction: the C oracle (bitwise
    the reference), so the rehearsal checks the protocol, not arithmetic."""
    import numpy as np
    import torch

    from oracle import ref

    ai = None if acc_in is None else np.ascontiguousarray(acc_in.numpy()).copy()
    res = ref.reduce(np.ascontiguousarray(X.numpy()), [float(v) for v in w32.tolist()],
                     acc_in=ai, W=W)
    out.copy_(torch.from_numpy(res))
    return out


def _oracle_step(step, avg):
    """Rehearsal stand-in for the HIP server step: the C oracle's."""
    from oracle import ref

    avg = avg.contiguous()
    a, g = step.args, step.sgd
    ref.lib().ref_server_step_f32(a.algo, avg.data_ptr(), a.coef, a.cloud, a.aux, a.avg_prev,
                                  a.momentum_buf, a.momentum_init, a.grad_out, g.neg_lr,
                                  g.momentum, g.one_minus_dampening, g.weight_decay, g.nesterov,
                                  g.maximize, step.P)


def _rehearsal_entry():
    """entry_factory of the aggregators in the CPU rehearsal: a rank's rows
    reduced by the C oracle (onto another rank's running sum for the chain)."""
    import torch

    from fedsim_amd import ops
    from fedsim_amd.utils.aggregators import _TensorEntry

    class Entry(_TensorEntry):
        def __init__(self, part, agg):
            self.P, self.dev, self.rows, self.ws, self.cur_w = part.numel(), part.device, [], [], 0

        def add(self, value, weight):
            new_w = self.cur_w + weight
            self.rows.append(value.detach().reshape(-1).clone())
            self.ws.append(weight)
            self.cur_w = new_w

        def partial(self, acc_in, W=None):
            out = torch.empty(self.P)
            w32 = torch.tensor([ops.fl32(w) for w in self.ws])
            return _oracle_reduce(torch.stack(self.rows), w32, out, acc_in, W)

        def get(self):
            return self.partial(None, self.cur_w if self.cur_w else None)

        def get_sum(self):
            return self.partial(None)

        def pop(self, on_device=False):
            return self.get()

        def pop_step(self, step):
            _oracle_step(step, self.get())

        def chainable(self):
            return True

    return Entry


def multi_gpu_selftest(rk, fault_rank=None, fault_devices=False):
    """One small round through every multi-GPU path over the job's real
    process group (RCCL on the GPUs; gloo in the rehearsal), each checked
    against the C oracle (oracle/ref.py) on every column: SURVEY §8e's
    decompositions of aggregators.py:23-40,104-122.

      sharded_pop_step    ShardedSerialAggregator: column shards, server step
                          on each, one all-gather of the operands   bitwise
      client_chain        ClientShardedSerialAggregator(mode="chain"): the
                          running sum passed rank to rank + broadcast  bitwise
      client_allreduce    mode="allreduce": partial sums + RCCL all-reduce
                          (reordered)                        normwise <= 1e-6
      client_bf16_key     a bf16 key in a client-sharded round: the
                          reference's arithmetic, chained as raw bytes
                          (vs oracle/reference_loop)                 bitwise
      param_sharded_step  sharding.param_sharded_step on this rank's column
                          shard (blocked slab, fused step)           bitwise
      devices_*           rank 0, when it sees > 1 GPU: the one-process
                          ShardedSerialAggregator(devices=[...]) on host /
                          pinned / HBM vectors, get / pop / momentum
                          pop_step with host and HBM clouds          bitwise

    Every rank checks its own result; the verdicts are combined with a MIN
    all-reduce, so every rank agrees.  Returns the dict that goes into the
    line as ``multi_gpu_selftest``."""
    import numpy as np
    import torch

    from fedsim_amd import ops, sharding
    from fedsim_amd.sharding import (ClientShardedSerialAggregator, RemoteRow,
                                     ShardedSerialAggregator)
    from oracle import ref
    from oracle import vectors as V

    t0 = time.perf_counter()
    K, P, world, me, dev = SELFTEST_K, SELFTEST_P, rk.world, rk.rank, rk.dev
    X = V.client_rows("realistic", K, P, 17)  # the same on every rank
    w = V.client_weights("fedavg", K, 17)
    W = sum(w)
    avg_ref = ref.reduce(X, w, W=W)
    cloud0 = V.cloud_vector(P, 18)
    cloud_ref = ref.fedavg_sgd(avg_ref, cloud0, 1.0)
    grad_ref = (cloud0 - avg_ref).astype(np.float32)
    entry = _rehearsal_entry() if rk.rehearsal else None
    kw = dict(entry_factory=entry) if entry is not None else {}
    checks = {}

    def record(name, got, want, bitwise=True):
        got = np.ascontiguousarray(got, dtype=np.float32)
        if bitwise:
            bad = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
            checks[name] = dict(bitwise=True, columns=int(want.size), mismatched=bad, ok=bad == 0)
        else:
            err = float(np.linalg.norm(got.astype(np.float64) - want) / np.linalg.norm(want))
            checks[name] = dict(bitwise=False, columns=int(want.size), rel_err=err,
                                tol=1e-6, ok=err <= 1e-6)

    def row(k):
        return torch.from_numpy(X[k].copy()).to(dev)

    # (1) parameter-sharded aggregator: pop + server step, all-gather
    agg = ShardedSerialAggregator(**kw)
    for k in range(K):
        agg.add("p", row(k), w[k])
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    grad = torch.empty_like(cloud)
    agg.pop_step("p", ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad))
    record("sharded_pop_step", cloud.cpu().numpy(), cloud_ref)
    record("sharded_pop_step_grad", grad.cpu().numpy(), grad_ref)
    # (2) client-sharded: each rank holds one contiguous block of the clients
    spans = [sharding.shard_range(K, r, world) for r in range(world)]
    owner = [next(r for r, (lo, hi) in enumerate(spans) if lo <= k < hi) for k in range(K)]
    for mode in ("chain", "allreduce"):
        agg = ClientShardedSerialAggregator(mode=mode, **kw,
                                            **(dict(step_impl=_oracle_step) if entry else {}))
        for k in range(K):
            v = row(k) if owner[k] == me else RemoteRow(
                (P,), torch.float32, "cpu" if rk.rehearsal else "cuda", owner[k])
            agg.add("p", v, w[k])
        record("client_" + mode, agg.pop("p").cpu().numpy(), avg_ref, bitwise=mode == "chain")
    # a bf16 key (a bf16 model's vectors) in the same client-sharded round:
    # the reference's arithmetic, its running sum chained rank to rank as raw
    # bytes (sharding._ClientShardRef), against the reference restatement
    from oracle.reference_loop import ReferenceSerialAggregator

    Xh = torch.from_numpy(X).to(torch.bfloat16)
    refagg = ReferenceSerialAggregator()
    agg = ClientShardedSerialAggregator(mode="allreduce", **kw,
                                        **(dict(step_impl=_oracle_step) if entry else {}))
    for k in range(K):
        refagg.add("h", Xh[k], w[k])
        v = Xh[k].to(dev) if owner[k] == me else RemoteRow(
            (P,), torch.bfloat16, "cpu" if rk.rehearsal else "cuda", owner[k])
        agg.add("h", v, w[k])
    got, want = agg.pop("h").cpu(), refagg.pop("h")
    bad = int((got.view(torch.int16) != want.view(torch.int16)).sum())
    checks["client_bf16_key"] = dict(bitwise=True, columns=P, mismatched=bad, ok=bad == 0)
    # (3) the parameter-sharded round step of bench's own headline mode
    lo, hi = sharding.shard_range(P, me, world, sharding.ALIGN)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    step = ops.ServerStep("fedavg", cloud, lr=1.0).narrow(lo, hi)
    if hi > lo:
        Xs = torch.from_numpy(np.ascontiguousarray(X[:, lo:hi])).to(dev)
        if rk.rehearsal:
            avg = sharding.param_sharded(Xs, w32, W, torch.empty(hi - lo),
                                         local_reduce=lambda *args: _oracle_reduce(*args[:5]))
            _oracle_step(step, avg)
        else:
            C = ops.choose_block_cols(hi - lo)
            sharding.param_sharded_step(ops.to_blocked(Xs, C), w32, W, step)
    got = cloud[lo:hi].cpu().numpy()
    if fault_rank == me:  # TEST ONLY: a wrong bit on one rank must fail every rank
        got = got.copy()
        got.view(np.uint32)[:1] ^= 1
    record("param_sharded_step", got, cloud_ref[lo:hi])
    # (4) the single-process multi-GPU mode (every local GPU, one process), on
    # rank 0 only, fenced by barriers so no collective of the others overlaps
    rk.barrier()
    devices = None
    if me == 0:
        devices = devices_selftest(rk, X, w, W, avg_ref, cloud0, record)
        if fault_devices:  # TEST ONLY: a failing devices_* check must fail every rank
            checks["devices_get_pageable"] = dict(bitwise=True, columns=P, mismatched=1,
                                                  ok=False, injected=True)
    rk.barrier()
    ok = all(c["ok"] for c in checks.values())
    if rk.dist is not None:  # every rank's verdict, agreed by all
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device="cpu" if rk.dist.get_backend() == "gloo" else dev)
        rk.dist.all_reduce(t, op=rk.dist.ReduceOp.MIN)
        ok = bool(t.item())
    if not rk.rehearsal:
        torch.cuda.synchronize()
    return dict(ok=ok, agreed="MIN of every rank's verdict (all-reduce)" if rk.dist else None,
                world=world, backend=rk.dist.get_backend() if rk.dist else None,
                K=K, P=P, seconds=round(time.perf_counter() - t0, 3),
                checker="oracle/ref.py (C restatement, pinned to the reference's goldens)",
                devices=(devices if devices is not None else
                         "rank 0: ShardedSerialAggregator(devices=%d local GPUs)"
                         % rk.torch.cuda.device_count()) if me == 0 else None,
                checks=checks)


def devices_selftest(rk, X, w, W, avg_ref, cloud0, record):
    """ShardedSerialAggregator(devices=[every local GPU]) -- the one-process
    multi-GPU mode FedSim's own simulator would use (one aggregator per round
    in one process, centralized_fl_algorithm.py:417-429) -- checked on rank 0
    against the C oracle, bitwise: get / pop with pageable, pinned and HBM
    client vectors, and a momentum SGD pop_step with the cloud on the host and
    in HBM.  Records ``devices_*`` checks; returns the skip reason (or None)."""
    import torch

    from fedsim_amd import ops
    from fedsim_amd.sharding import ShardedSerialAggregator

    if rk.rehearsal:
        return "skipped: no HIP device (CPU rehearsal)"
    n = torch.cuda.device_count()
    if n < 2:
        return "skipped: 1 device"
    devs = list(range(n))
    K, P = X.shape
    src = {"pageable": lambda k: torch.from_numpy(X[k].copy()),
           "pinned": lambda k: torch.from_numpy(X[k].copy()).pin_memory(),
           "hbm": lambda k: torch.from_numpy(X[k].copy()).to(rk.dev)}
    for name, make in src.items():
        agg = ShardedSerialAggregator(devices=devs)
        for k in range(K):
            agg.add("p", make(k), w[k])
        got = agg.get("p")
        record("devices_get_" + name, got.cpu().numpy(), avg_ref)
        record("devices_pop_" + name, agg.pop("p").cpu().numpy(), avg_ref)
    # momentum SGD (lr 0.5, momentum 0.9, weight decay 1e-3; first step: the
    # buffer is initialised from the gradient), oracle on host copies
    kw = dict(lr=0.5, momentum=0.9, weight_decay=1e-3)
    c_ref = torch.from_numpy(cloud0.copy())
    b_ref = torch.zeros(P)
    g_ref = torch.empty(P)
    _oracle_step(ops.ServerStep("fedavg", c_ref, momentum_buf=b_ref, momentum_init=True,
                                grad_out=g_ref, **kw), torch.from_numpy(avg_ref.copy()))
    for where in ("host", "hbm"):
        on = torch.device("cpu") if where == "host" else rk.dev
        agg = ShardedSerialAggregator(devices=devs)
        for k in range(K):
            agg.add("p", src["hbm" if where == "hbm" else "pageable"](k), w[k])
        cloud = torch.from_numpy(cloud0.copy()).to(on)
        buf = torch.zeros(P, device=on)
        grad = torch.empty(P, device=on)
        agg.pop_step("p", ops.ServerStep("fedavg", cloud, momentum_buf=buf, momentum_init=True,
                                         grad_out=grad, **kw))
        record("devices_pop_step_%s_cloud" % where, cloud.cpu().numpy(), c_ref.numpy())
        record("devices_pop_step_%s_momentum" % where, buf.cpu().numpy(), b_ref.numpy())
        record("devices_pop_step_%s_grad" % where, grad.cpu().numpy(), g_ref.numpy())
    torch.cuda.synchronize()
    return None


def fedavg_step(rk, P):
    """FedAvg.optimize's server step operands (default SGD lr 1.0,
    fed_learn.py:129; cloud.grad = pseudo-gradient as torch leaves it)."""
    from fedsim_amd import ops

    torch = rk.torch
    cloud = torch.zeros(P, dtype=torch.float32, device=rk.dev)
    grad = torch.empty(P, dtype=torch.float32, device=rk.dev)
    return ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=grad), cloud, grad


# -- driver-timed side legs (rank 0 at N=1, after the headline) -------------
H2D_K, H2D_POOL = 64, 8


def _sample_cols(P, n=4096, seed=5):
    import numpy as np

    cols = np.random.default_rng(seed).integers(0, P, size=n)
    return np.unique(np.concatenate([cols, np.arange(max(0, P - 64), P)]))


def h2d_inclusive_leg(rk, P, repeats=3):
    """The round the north star names second: client vectors arrive as HOST
    tensors (the reference's CPU-side trainers) and the average returns to
    the host -- ``SerialAggregator(borrow_host=True).add`` x K then ``pop``
    into a host tensor, wall clock (perf_counter around synchronised rounds),
    once from pageable and once from pinned vectors (a pool of H2D_POOL
    distinct 4P-byte tensors cycled over K adds: PCIe-bound, host memory is
    read once per client either way).  The PCIe ceiling is one plain pinned
    H2D copy of the same bytes in this process.  The popped average is
    checked bitwise against the C oracle on sampled columns, outside the
    timing.  Reference: training/utils.py:34 (the clone), aggregators.py:
    23-40, 104-122."""
    import numpy as np
    import torch

    from fedsim_amd.utils import SerialAggregator
    from oracle import ref

    K = H2D_K
    weights = _weights(K, seed=13)
    W = sum(weights)
    g = torch.Generator().manual_seed(29)
    base = torch.empty(P).normal_(0.0, 0.05, generator=g)
    pageable = [base + float(k) * 1e-3 for k in range(H2D_POOL)]
    pinned = [t.pin_memory() for t in pageable]
    cols = _sample_cols(P)
    want = ref.reduce(np.stack([pageable[k % H2D_POOL].numpy()[cols] for k in range(K)]),
                      weights, W=W)

    def one_round(pool):
        agg = SerialAggregator(borrow_host=True, expected_rows=K)
        for k in range(K):
            agg.add("local_params", pool[k % H2D_POOL], weights[k])
        return agg.pop("local_params")  # host tensor: the D2H completes here

    res = dict(K=K, P=P, pool=H2D_POOL, repeats=repeats, bytes_per_round=4.0 * K * P)
    checked = True
    for name, pool in (("pageable", pageable), ("pinned", pinned)):
        out = one_round(pool)  # warm (ingest ring, staging slots, slab)
        got = out.numpy()[cols]
        checked &= bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        secs = []
        for _ in range(repeats):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = one_round(pool)
            torch.cuda.synchronize()
            secs.append(time.perf_counter() - t0)
        assert out.device.type == "cpu"
        res[name] = round(4.0 * K * P / (sum(secs) / len(secs)) / 1e9, 2)
        res[name + "_ms"] = round(sum(secs) / len(secs) * 1e3, 2)
    dst = torch.empty(P, device=rk.dev)
    dst.copy_(pinned[0], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        dst.copy_(pinned[k % H2D_POOL], non_blocking=True)
    torch.cuda.synchronize()
    res["ceiling"] = round(4.0 * K * P / (time.perf_counter() - t0) / 1e9, 2)
    res["ratio"] = {n: round(res[n] / res["ceiling"], 3) for n in ("pageable", "pinned")}
    res["checked"] = checked
    res["unit"] = "GB/s"
    res["check"] = "popped average vs oracle/ref.reduce on %d sampled columns, bitwise" % cols.size
    res["ceiling_is"] = "plain pinned H2D copies of the same 4KP bytes (torch copy_, one stream)"
    return res


CONFIG_P = 1_085_668  # SimpleCNN2 on CIFAR-100 (BASELINE configs 2 and 3)
CONFIG_LEGS = (("cfg2_fedavg_K1000", "fedavg", 1000), ("cfg2_fedavg_K10", "fedavg", 10),
               ("cfg3_adabest_K1000", "adabest", 1000), ("cfg3_adabest_K10", "adabest", 10))


def config_legs(rk, steps=20, warmup=2):
    """BASELINE configs 2 and 3 on the device-resident path: one server
    round of K client rows of SimpleCNN2 (P = 1,085,668) packed in the
    column-blocked slab, the exact reduce + divide and the server step --
    FedAvg (lr 1.0, weights = sample counts U{50..600}) and AdaBest (beta 0.6,
    lr 1.0, weight 1 per client, avg_params in place) -- through the library's
    own pop_step policy (_DeviceEntry.pop_step: fused into the last pass when
    ops.fuse_step_pays, else reduce then fedagg_server_step_f32).  Each is
    checked first, one round from a known state, against oracle/ref on
    sampled columns (bitwise), then timed over ``steps`` rounds with HIP
    events.  Reference: fedavg.py:193-208, adabest.py:172-189."""
    import numpy as np
    import torch

    from fedsim_amd import ops
    from oracle import ref

    P = CONFIG_P
    C = ops.choose_block_cols(P)
    cols = _sample_cols(P)
    cols_t = torch.from_numpy(cols).to(rk.dev)
    out = {}
    for name, algo, K in CONFIG_LEGS:
        Xb = make_pool(rk, K, P, C, seed=41 + K)
        weights = _weights(K, seed=17) if algo == "fedavg" else [1] * K
        W = sum(weights)
        w32 = torch.tensor([ops.fl32(v) for v in weights], dtype=torch.float32, device=rk.dev)
        g = torch.Generator(device=rk.dev).manual_seed(43)
        cloud = torch.empty(P, device=rk.dev).normal_(0.0, 0.05, generator=g)
        aux = torch.empty(P, device=rk.dev).normal_(0.0, 0.05, generator=g) \
            if algo == "adabest" else None
        grad = torch.empty(P, device=rk.dev)
        avg = torch.empty(P, device=rk.dev)
        step = ops.ServerStep(algo, cloud, lr=1.0, coef=0.6 if algo == "adabest" else 0.0,
                              aux=aux, grad_out=grad)
        fused = ops.can_fuse_step(Xb, step) and ops.fuse_step_pays(P, K)

        def one_round():
            if fused:
                ops.reduce_blocked_step(Xb, w32, step, W=W)
            else:
                ops.reduce_blocked(Xb, w32, avg, W=W, flags=ops.default_flags(C))
                step.apply(avg)

        c0 = cloud[cols_t].cpu().numpy()
        a0 = aux[cols_t].cpu().numpy() if aux is not None else None
        Xs = Xb[cols_t // C, :, cols_t % C].T.contiguous().cpu().numpy()  # [K, cols]
        one_round()
        avg_ref = ref.reduce(Xs, weights, W=W)
        if algo == "fedavg":
            want = dict(cloud=ref.fedavg_sgd(avg_ref, c0, 1.0))
        else:
            c_ref, ap_ref = ref.adabest_sgd(avg_ref, c0, a0, 0.6, 1.0)
            want = dict(cloud=c_ref, aux=ap_ref)
        got = dict(cloud=cloud[cols_t].cpu().numpy())
        if aux is not None:
            got["aux"] = aux[cols_t].cpu().numpy()
        checked = all(np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32))
                      for k in want)
        for _ in range(warmup):
            one_round()
        marks = []
        for _ in range(steps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            one_round()
            e1.record()
            marks.append((e0, e1))
        torch.cuda.synchronize()
        ms = sum(e0.elapsed_time(e1) for e0, e1 in marks) / steps
        # algorithmic bytes: client rows + weights + per column the step's
        # operands (cloud r/w, grad w; AdaBest's avg_params r/w) and, split,
        # the stored average's write + read
        per_col = 12.0 + (8.0 if algo == "adabest" else 0.0) + (0.0 if fused else 8.0)
        alg = 4.0 * K * P + 4.0 * K + per_col * P
        out[name] = dict(algo=algo, K=K, P=P, C=C, weights="sample counts U{50..600}"
                         if algo == "fedavg" else "1 per client", lr=1.0,
                         beta=0.6 if algo == "adabest" else None,
                         path="fused" if fused else "split", steps=steps,
                         ms=round(ms, 4), GBps=round(4.0 * K * P / ms / 1e6, 1),
                         alg_bytes=alg, frac=round(alg / ms / 1e6 / PEAK_HBM_GBPS, 4),
                         checked=checked,
                         check="%d sampled columns vs oracle/ref, bitwise (%s)" % (
                             cols.size, ", ".join(sorted(want))))
        del Xb
    return out


# -- param: the headline round ---------------------------------------------
def setup_param(a, rk, clock):
    from fedsim_amd import ops

    torch = rk.torch
    K, P = a.K, a.P
    X = make_inputs(rk, K, P, a.layout, a.C)
    weights = _weights(K)
    W = sum(weights)
    w32 = torch.tensor([ops.fl32(v) for v in weights], dtype=torch.float32, device=rk.dev)
    info = dict(clients_K=K, params_per_gpu_P=P, params_total=P * rk.world,
                parallelism=f"param-shard{rk.world}" if rk.world > 1 else "single",
                mode="exact (bitwise vs reference CPU)")
    if rk.rehearsal:
        out = torch.empty(P)
        info["layout"] = "row-major (rehearsal)"

        def step():
            rk.stub(X[:, :P], w32, out, None, W)
        return step, info, 4.0 * K * P * rk.world, (X,)

    flags = ops.tuning_flags(unroll=a.unroll, vpt=a.vpt if a.layout == "strided" else 0,
                             nt=bool(a.nt), mapping=a.mapping)
    fused = a.step == "fused" and a.layout == "blocked" and not a.no_epilogue
    avg = torch.empty(P, dtype=torch.float32, device=rk.dev)
    sstep, cloud, grad = fedavg_step(rk, P)
    # client rows + weights, plus per column: fused = cloud read + cloud write +
    # grad write; split (reduce kernel alone) = the average's write
    nbytes = 4.0 * K * P + 4.0 * K + (12.0 * P if fused else 4.0 * P)

    def reduce():
        if fused:
            ops.reduce_blocked_step(X, w32, sstep, W=W, mapping=a.mapping)
        elif a.layout == "strided":
            ops.reduce_slab(X[:, :P], w32, avg, W=W, P=P, flags=flags)
        else:
            ops.reduce_blocked(X, w32, avg, W=W, flags=flags)

    def step():
        clock.run(nbytes, reduce)
        if not a.no_epilogue and not fused:
            ops.fedavg_sgd(avg, cloud, 1.0, grad_out=grad)

    mapping, unroll = ops.column_mapping(
        P, ops.tuning_flags(mapping=a.mapping) if fused else flags, B=K)
    kernel = ("k_reduce_vec" if mapping == "wide" else
              f"k_reduce_narrow<U={unroll}, VW={mapping[-1]}>")
    step_mode = "fused" if fused else "split"
    info.update(
        workload=("FedAvg server round, device-resident: exact weighted reduce + divide "
                  "+ SGD server step in one pass" if fused else
                  "FedAvg server round, device-resident: exact weighted reduce + divide, "
                  "then the SGD epilogue kernel"),
        step=step_mode,
        layout=a.layout if a.layout == "strided" else f"blocked C={a.C}",
        mapping=mapping if mapping == "wide" else f"{mapping} (U={unroll})",
        flags=flags)
    info["_kernel"] = "%s (%s)" % (kernel,
        "fedagg_reduce_step_blocked_f32, EpiStep<FEDAVG>" if fused else
        "fedagg_reduce_blocked_f32" if a.layout == "blocked" else "fedagg_reduce_f32")
    from fedsim_amd import _native

    info["_traffic"] = load_pmc(a.pmc_json, K, P, kernel,
                                a.layout if a.layout == "strided" else f"blocked{a.C}",
                                step_mode, _native.LIB_PATH)
    return step, info, 4.0 * K * P * rk.world, (X, avg, cloud, grad)


# -- streamed rounds (strong / allreduce) ----------------------------------
def _pool_rows(a, rk, K, P, C):
    """Resident rows: --pool-rows, else (allreduce) 200, else (strong) as many
    of the K rows as fit the free HBM less 16 GiB of headroom."""
    if a.pool_rows:
        return min(K, a.pool_rows)
    if a.mode == "allreduce":
        return min(K, 200)
    if rk.rehearsal:
        return K
    row_bytes = 4 * ((P + C - 1) // C) * C
    free, _ = rk.torch.cuda.mem_get_info(rk.dev)
    fit = max(1, (free - (16 << 30) - 4 * 4 * P) // row_bytes)
    return int(min(K, fit))


def setup_streamed(a, rk, clock):
    """strong: this rank's column shard of all K clients; allreduce: all P
    columns of this rank's K clients, then all-reduce of the partial sum.
    Rows beyond the resident pool are re-reads of it (accumulator chained
    through acc_in: +8P bytes per extra pass, not counted as algorithmic)."""
    from fedsim_amd import ops, sharding

    torch = rk.torch
    if a.mode == "strong":
        lo, hi = sharding.shard_range(a.P, rk.rank, rk.world, sharding.ALIGN)
        P, K, K_total = hi - lo, a.K, a.K
        weights = _weights(K)
        W = sum(weights)
    else:
        P, K, K_total = a.P, a.K, a.K * rk.world
        all_w = _weights(K_total)
        weights = all_w[rk.rank * K:(rk.rank + 1) * K]
        W = sum(all_w)  # the host sums the weights of every rank's clients
    C = ops.choose_block_cols(P)
    R = _pool_rows(a, rk, K, P, C)
    counts = [min(R, K - k0) for k0 in range(0, K, R)]
    pool = make_pool(rk, R, P, C, seed=3 + rk.rank)
    w32 = torch.tensor([ops.fl32(v) for v in weights], dtype=torch.float32, device=rk.dev)
    acc = torch.empty(P, dtype=torch.float32, device=rk.dev)
    ar_ms = []
    info = dict(clients_K=K_total, params_per_gpu_P=P, params_total=a.P,
                pool_rows=R, passes=len(counts),
                pool_GB=round(4.0 * R * P / 1e9, 1))
    if rk.rehearsal:
        info["layout"] = "row-major (rehearsal)"

        def step():
            for i, n in enumerate(counts):
                last = i == len(counts) - 1
                rk.stub(pool[:n], w32[i * R:i * R + n], acc, None if i == 0 else acc,
                        W if (last and a.mode == "strong") else None)
            if a.mode == "allreduce":
                if rk.dist is not None:
                    rk.dist.all_reduce(acc)
                acc.div_(ops.fl32(W))
        info.update(parallelism=("param-shard%d" % rk.world if a.mode == "strong"
                                 else "client-shard%d+allreduce" % rk.world))
        total = 4.0 * K * (a.P if a.mode == "strong" else P * rk.world)
        return step, info, total, (pool,), ar_ms

    sstep, cloud, grad = fedavg_step(rk, P)
    flags = ops.default_flags(C)
    fuse_last = a.mode == "strong"  # allreduce: the step needs the global sum

    def one_pass(i, n, last):
        wv = w32[i * R:i * R + n]
        acc_in = None if i == 0 else acc
        if last and fuse_last:
            nb = 4.0 * n * P + 4.0 * n + 12.0 * P
            clock.run(nb, lambda: ops.reduce_blocked_step(pool, wv, sstep, B=n, acc_in=acc_in,
                                                          W=W))
        else:
            nb = 4.0 * n * P + 4.0 * n + 4.0 * P
            clock.run(nb, lambda: ops.reduce_blocked(pool, wv, acc, B=n, acc_in=acc_in,
                                                     flags=flags))

    def step():
        for i, n in enumerate(counts):
            one_pass(i, n, i == len(counts) - 1)
        if a.mode == "allreduce":
            if rk.dist is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                rk.dist.all_reduce(acc, op=rk.dist.ReduceOp.SUM)
                e1.record()
                if clock.on:
                    ar_ms.append((e0, e1))
            ops.finalize(acc, W, out=acc)
            sstep.apply(acc)

    kname = "k_reduce_narrow (fedagg_reduce_blocked_f32 passes%s)" % (
        " + fedagg_reduce_step_blocked_f32 last pass" if fuse_last else "")
    info.update(
        workload=("FedAvg server round, parameter-sharded (config 4): this rank's column "
                  "shard of every client, exact reduce + divide + SGD step fused into "
                  "the last pass" if a.mode == "strong" else
                  "FedAvg server round, client-sharded (config 5): this rank's clients "
                  "reduced in order into a partial sum, RCCL all-reduce(sum) of 4P bytes, "
                  "divide by fl32(W), SGD server step"),
        parallelism=("param-shard%d" % rk.world if a.mode == "strong"
                     else "client-shard%d+allreduce" % rk.world),
        mode=("exact (bitwise vs reference CPU)" if a.mode == "strong"
              else "reordered across ranks (normwise <= 1e-6 vs reference CPU)"),
        layout=f"blocked C={C}", step="fused" if fuse_last else "split")
    info["_kernel"] = kname
    info["_traffic"] = (None, dict(reason="no PMC summary is kept for the streamed modes"))
    total = 4.0 * K * (a.P if a.mode == "strong" else P * rk.world)
    return step, info, total, (pool, acc, cloud, grad), ar_ms


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a, argv))
    quiet = _StdoutToStderr()
    try:
        _main(a, quiet)
    finally:
        quiet.restore()


def _main(a, quiet):
    rk = Rank(a)
    if a.gpus != rk.world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={rk.world}")
    clock = KernelClock(rk)
    ar_ms = []
    selftest = None if a.no_selftest else multi_gpu_selftest(rk, a.selftest_fault_rank,
                                                             a.selftest_fault_devices)
    if a.mode == "param":
        step, info, total_bytes, keep = setup_param(a, rk, clock)
    else:
        step, info, total_bytes, keep, ar_ms = setup_streamed(a, rk, clock)

    for _ in range(a.warmup):
        step()
    rk.sync()
    clock.on = True
    rk.barrier()
    rk.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    rk.sync()
    rk.barrier()
    elapsed = time.perf_counter() - t0
    clock.on = False
    nbytes, kern_ms = clock.summary()
    ar = None
    if ar_ms:
        ar = sum(e0.elapsed_time(e1) for e0, e1 in ar_ms) / len(ar_ms)
    elapsed, kern_ms_max, ar_max = rk.max_over_ranks(
        elapsed, kern_ms if kern_ms is not None else 0.0, ar if ar is not None else 0.0)

    value = total_bytes * a.steps / elapsed / 1e9
    kernel = info.pop("_kernel", None)
    traffic, traffic_source = info.pop("_traffic", (None, None))
    result = {
        "metric": METRIC,
        "value": float(f"{value:.6g}"),  # 6 significant digits: tiny rehearsals stay > 0
        "unit": "GB/s",
        "n_gpus": rk.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.mode == "strong" else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (x_k = base + eps_k on device, FedAvg int weights U{50..600})"
                 if a.mode == "param" else
                 "synthetic (resident pool of distinct N(0, 0.05) client rows, re-read "
                 "cyclically; FedAvg int weights U{50..600})"),
        "config": dict(info, mode_flag=a.mode),
    }
    result["multi_gpu_selftest"] = selftest
    result["world_size_seen"] = rk.dist.get_world_size() if rk.dist is not None else 1
    result["backend"] = rk.dist.get_backend() if rk.dist is not None else None
    if rk.rehearsal:
        result["rehearsal"] = "cpu/gloo launcher rehearsal, per-rank reduce = " + a.rehearsal_stub
        result["roofline"] = None
    else:
        if a.one_gpu_rehearsal:
            result["rehearsal"] = ("one-GPU launcher rehearsal: %d ranks share cuda:0 over "
                                   "gloo (not a scaling number)" % rk.world)
        achieved = nbytes / (kern_ms_max * 1e-3) / 1e9
        result["roofline"] = {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "launch_ms": round(kern_ms_max, 4),
            "alg_bytes_per_launch": nbytes,
        }
        if a.mode == "allreduce":
            result["allreduce"] = dict(
                ms=round(ar_max, 4) if ar_ms else None,
                bytes=4 * a.P,
                share_of_round=round(ar_max / (elapsed / a.steps * 1e3), 4) if ar_ms else None,
                note="RCCL all-reduce(sum) of the fp32 partial, HIP events on the compute "
                     "stream around the call (max over ranks); none at N=1 without a "
                     "process group")
    del keep, step
    if not rk.rehearsal:
        rk.torch.cuda.empty_cache()
    if rk.rank == 0 and rk.world == 1 and not rk.rehearsal and a.mode == "param" \
            and not a.no_side_legs:
        t0 = time.perf_counter()
        result["h2d_inclusive"] = h2d_inclusive_leg(rk, a.P)
        result["configs"] = config_legs(rk)
        result["side_legs_s"] = round(time.perf_counter() - t0, 2)
        rk.torch.cuda.empty_cache()
    if rk.rank == 0 and rk.world == 1 and not a.no_cpu_baseline and not rk.rehearsal:
        result["cpu_baseline"] = cpu_baseline(a.P, a.cpu_baseline_seconds)
    if rk.rank == 0:
        quiet.restore()
        print(json.dumps(result), flush=True)
    if rk.dist is not None:
        rk.dist.barrier()
        rk.dist.destroy_process_group()
    if selftest is not None and not selftest["ok"]:
        sys.stderr.write("bench: multi-GPU self-test FAILED: %s\n" % json.dumps(selftest))
        sys.exit(3)


if __name__ == "__main__":
    main()
