"""Multi-process (world_size 2 and 3) CPU rehearsal of the multi-GPU protocols
in fedsim_amd.sharding over the gloo backend.  The per-rank reduction is the
C oracle injected as ``local_reduce`` (no GPU here); what is tested is the
decomposition, the collectives and the ordering guarantees:
  param     concatenated shards == single-device reference, bitwise
  chain     client-sharded pipeline == single-device reference, bitwise
  allreduce client-sharded partial sums: normwise <= 1e-6 + forward-error bound
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import bits
from oracle import ref
from oracle import vectors as V


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def oracle_reduce(X, w32, out, acc_in, W, flags):
    """CPU stand-in for the HIP kernel (same bits)."""
    Xn = np.ascontiguousarray(X.numpy())
    ai = None if acc_in is None else np.ascontiguousarray(acc_in.numpy()).copy()
    res = ref.reduce(Xn, [float(v) for v in w32.tolist()], acc_in=ai, W=W)
    out.copy_(torch.from_numpy(res))
    return out


def _worker(rank, world, port, K, P, mode, outdir):
    import torch.distributed as dist

    from fedsim_amd import sharding

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X = torch.from_numpy(V.client_rows("normal", K, P, 21))
        w = V.client_weights("fedavg", K, 21)
        W = sum(w)
        if mode == "param":
            lo, hi = sharding.shard_range(P, rank, world, sharding.ALIGN)
            out = torch.empty(hi - lo)
            sharding.param_sharded(X[:, lo:hi], sharding.weights_fp32(w, "cpu"), W, out,
                                   local_reduce=oracle_reduce)
            # assemble on rank 0 for checking (not part of the data path)
            sizes = [sharding.shard_range(P, r, world, sharding.ALIGN) for r in range(world)]
            parts = [torch.empty(h - l_) for l_, h in sizes]
            if rank == 0:
                parts[0] = out
                for r in range(1, world):
                    dist.recv(parts[r], src=r)
            else:
                dist.send(out, dst=0)
            res = torch.cat(parts) if rank == 0 else None
        else:
            klo, khi = sharding.shard_range(K, rank, world)
            Xl = X[klo:khi].contiguous()
            wl = sharding.weights_fp32(w[klo:khi], "cpu")
            res = torch.empty(P)
            if mode == "chain":
                sharding.client_sharded_chain(Xl, wl, W, res, n_blocks=7,
                                              local_reduce=oracle_reduce)
            else:
                sharding.client_sharded_allreduce(Xl, wl, W, res, local_reduce=oracle_reduce)
        if res is not None:
            np.save(os.path.join(outdir, f"res{rank}.npy"), res.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["param", "chain", "allreduce"])
def test_sharded_protocols(mode, world):
    K, P = 23, 4099
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), K, P, mode, d), nprocs=world,
                           join=True, start_method="spawn")
        X = V.client_rows("normal", K, P, 21)
        w = V.client_weights("fedavg", K, 21)
        exp = ref.reduce(X, w, W=sum(w))
        got = np.load(os.path.join(d, "res0.npy"))
        if mode in ("param", "chain"):
            np.testing.assert_array_equal(bits(got), bits(exp))
            if mode == "chain":
                for r in range(1, world):
                    np.testing.assert_array_equal(
                        bits(np.load(os.path.join(d, f"res{r}.npy"))), bits(exp))
        else:
            x64 = X.astype(np.float64)
            w64 = np.array([np.float32(v) for v in w], dtype=np.float64)
            y64 = (w64[:, None] * x64).sum(0) / np.float64(np.float32(sum(w)))
            rel = np.linalg.norm(got - exp) / np.linalg.norm(exp)
            assert rel <= 1e-6
            gamma = K * 2.0 ** -24 / (1 - K * 2.0 ** -24)
            bound = (gamma * (np.abs(w64[:, None] * x64).sum(0)) / np.float32(sum(w))
                     + np.abs(y64) * 2.0 ** -23)
            assert np.all(np.abs(got.astype(np.float64) - y64) <= bound)


def test_shard_range_covers_and_aligns():
    from fedsim_amd.sharding import shard_range

    for n in (0, 1, 63, 64, 65, 1000, 25_000_000, 25_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world, 64) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
                assert b % 64 == 0 or b == n
