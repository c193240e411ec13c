"""bench.py's own N-rank launcher (``--gpus N`` without torch.distributed.run),
rehearsed on CPU over gloo with a stub per-rank reduction
(tests/bench_stub.py): exactly ONE JSON line on stdout, from rank 0, carrying
n_gpus = N; every mode; a failing rank fails the whole run instead of hanging
it.  The GPU run of the same launcher is in tests/test_gpu_bench.py."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args],
                          cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("mode", ["param", "strong", "allreduce"])
@pytest.mark.parametrize("gpus", [2, 3])
def test_launcher_one_line(mode, gpus):
    r = _bench("--gpus", str(gpus), "--mode", mode, "--rehearsal-stub",
               "tests.bench_stub:reduce", "--K", "9", "--P", "1000", "--steps", "2",
               "--warmup", "1", "--pool-rows", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus
    assert d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == ("strong" if mode == "strong" else "weak")
    assert d["config"]["mode_flag"] == mode
    if mode == "strong":
        assert d["config"]["params_total"] == 1000
    if mode == "allreduce":
        assert d["config"]["clients_K"] == 9 * gpus
    assert d["value"] > 0
    _selftest_ok(d, gpus)


SELFTEST_CHECKS = {"sharded_pop_step", "sharded_pop_step_grad", "client_chain",
                   "client_allreduce", "client_bf16_key", "param_sharded_step"}


def _selftest_ok(d, world):
    """The line carries the multi-GPU self-test: every path checked against
    the oracle over the job's process group, agreed by every rank."""
    st = d["multi_gpu_selftest"]
    assert st["ok"] and st["world"] == world, st
    assert set(st["checks"]) == SELFTEST_CHECKS
    # rank 0's one-process devices=[...] check needs several GPUs: recorded skip
    assert st["devices"] == "skipped: no HIP device (CPU rehearsal)"
    for name, c in st["checks"].items():
        assert c["ok"], (name, c)
        assert c["bitwise"] == (name != "client_allreduce")


def test_selftest_mismatch_fails_every_rank():
    """A wrong bit on one rank's shard: every rank agrees the self-test
    failed, the line says so, and the run exits non-zero."""
    r = _bench("--gpus", "3", "--rehearsal-stub", "tests.bench_stub:reduce", "--K", "4",
               "--P", "256", "--steps", "1", "--warmup", "1", "--selftest-fault-rank", "2",
               timeout=180)
    assert r.returncode == 3, r.stderr[-2000:]
    assert "multi-GPU self-test FAILED" in r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    st = json.loads(lines[0])["multi_gpu_selftest"]
    assert st["ok"] is False and st["checks"]["param_sharded_step"]["ok"] is True  # rank 0's


@pytest.mark.parametrize("gpus", [1, 3])
def test_selftest_devices_failure_fails_every_rank(gpus):
    """A failing devices_* check (rank 0's one-process multi-GPU mode, injected
    here since the rehearsal has no GPU) fails the self-test on every rank:
    the run exits 3 instead of timing, the line names the check."""
    r = _bench("--gpus", str(gpus), "--rehearsal-stub", "tests.bench_stub:reduce", "--K", "4",
               "--P", "256", "--steps", "1", "--warmup", "1", "--selftest-fault-devices",
               timeout=180)
    assert r.returncode == 3, r.stderr[-2000:]
    assert "multi-GPU self-test FAILED" in r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    st = json.loads(lines[0])["multi_gpu_selftest"]
    assert st["ok"] is False and st["checks"]["devices_get_pageable"]["ok"] is False
    assert all(c["ok"] for n, c in st["checks"].items() if not n.startswith("devices_"))


def test_launcher_rank_failure_fails_run():
    r = _bench("--gpus", "2", "--rehearsal-stub", "tests.bench_stub:fail_on_rank1", "--K", "4",
               "--P", "256", "--steps", "1", "--warmup", "1", timeout=120)
    assert r.returncode != 0
    assert "injected failure on rank 1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_mismatch_rejected():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--rehearsal-stub", "tests.bench_stub:reduce", "--K", "2", "--P", "64"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("mode", ["param", "strong", "allreduce"])
def test_driver_command_at_8_ranks(mode):
    """The driver's own 8-GPU form, rehearsed on CPU/gloo: torch.distributed.run
    --nproc-per-node 8 --master-addr 127.0.0.1 --master-port P bench.py --gpus 8.
    Exactly one JSON line (rank 0's), world_size_seen 8, n_gpus 8, the
    mode's scaling and decomposition (readiness)."""
    port = _free_port()
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(REPO, "bench.py"), "--gpus", "8", "--mode", mode,
                        "--rehearsal-stub", "tests.bench_stub:reduce", "--K", "9", "--P", "1000",
                        "--steps", "2", "--warmup", "1", "--pool-rows", "4"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["world_size_seen"] == 8
    assert d["scaling"] == ("strong" if mode == "strong" else "weak")
    assert d["backend"] == "gloo"
    if mode == "allreduce":  # (the all-reduce's HIP-event share: tests/test_gpu_bench.py)
        assert d["config"]["clients_K"] == 9 * 8
        assert d["config"]["parallelism"] == "client-shard8+allreduce"
    if mode == "strong":
        assert d["config"]["params_total"] == 1000
    assert "cpu_baseline" not in d or d["cpu_baseline"] is None  # rank 0 at N=1 only
    _selftest_ok(d, 8)
