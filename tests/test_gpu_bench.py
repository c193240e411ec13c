"""bench.py's own N-rank launcher with the HIP kernels: two ranks started by
``bench.py --gpus 2`` itself, both on the one GPU of the box over a gloo group
(``--one-gpu-rehearsal``; the 8-GPU RCCL run is the driver's), every mode:
exactly one JSON line on stdout with n_gpus 2, the world size the ranks saw,
and a roofline measured by each rank's HIP events."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode,extra", [
    ("param", ["--K", "64", "--P", "2000000"]),
    ("strong", ["--K", "300", "--P", "2000000", "--pool-rows", "128"]),
    ("allreduce", ["--K", "300", "--P", "2000000", "--pool-rows", "128"]),
])
def test_launcher_two_ranks_one_gpu(mode, extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--mode",
                        mode, "--one-gpu-rehearsal", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", *extra],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and d["backend"] == "gloo"
    assert d["roofline"]["achieved"] > 0 and d["roofline"]["launch_ms"] > 0
    assert "rehearsal" in d
    if mode == "allreduce":
        assert d["allreduce"]["ms"] is not None
    _selftest_ok(d, 2, "gloo")


def _selftest_ok(d, world, backend):
    from test_bench_launcher import SELFTEST_CHECKS

    st = d["multi_gpu_selftest"]
    assert st["ok"] and st["world"] == world and st["backend"] == backend, st
    assert set(st["checks"]) == SELFTEST_CHECKS and all(c["ok"] for c in st["checks"].values())


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("launch", ["plain", "torchrun_rccl"])
def test_one_gpu_line_carries_selftest(launch):
    """N=1 as the driver runs it (plain) and under torch.distributed.run
    with one rank (the RCCL process-group path): the HIP aggregators'
    multi-GPU paths checked against the oracle before the timed region."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    args = [os.path.join(REPO, "bench.py"), "--gpus", "1", "--K", "64", "--P", "2000000",
            "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    if launch == "torchrun_rccl":
        args = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    r = subprocess.run([sys.executable, *args], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    _selftest_ok(d, 1, "nccl" if launch == "torchrun_rccl" else None)
    # one GPU on the box: rank 0's devices=[...] check records its skip
    assert d["multi_gpu_selftest"]["devices"] == "skipped: 1 device"
    # the N=1 side legs: the host-to-host round and BASELINE configs 2 / 3,
    # each checked against the oracle before it is timed
    h = d["h2d_inclusive"]
    assert h["checked"] is True and h["P"] == 2_000_000 and h["K"] == 64
    assert 0 < h["pageable"] and 0 < h["pinned"] and 0 < h["ceiling"]
    cfg = d["configs"]
    assert set(cfg) == {"cfg2_fedavg_K1000", "cfg2_fedavg_K10", "cfg3_adabest_K1000",
                        "cfg3_adabest_K10"}
    for name, c in cfg.items():
        assert c["checked"] is True and c["ms"] > 0 and 0 < c["frac"] < 1.2, (name, c)
    assert cfg["cfg2_fedavg_K1000"]["path"] == "split"  # ops.fuse_step_pays at 1.09 M x 1000
    assert cfg["cfg2_fedavg_K10"]["path"] == "fused"
