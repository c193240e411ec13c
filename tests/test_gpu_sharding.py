"""The multi-GPU protocols of fedsim_amd.sharding with the real HIP per-rank
reducer, on a one-rank RCCL ("nccl") process group (the 8-GPU run belongs to the
driver).  Bit-exact vs the oracle for param / chain; the all-reduce path must
still be exact at one rank (nothing is reordered)."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist

    if dist.is_initialized():
        yield dist
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["param", "chain", "allreduce"])
def test_sharding_protocols_one_rank(mode, pg):
    from fedsim_amd import sharding

    dev = torch.device("cuda", 0)
    K, P = 37, 100_003
    X = V.client_rows("normal", K, P, 9)
    w = V.client_weights("fedavg", K, 9)
    W = sum(w)
    exp = ref.reduce(X, w, W=W)
    Xd = torch.from_numpy(X).to(dev)
    w32 = sharding.weights_fp32(w, dev)
    out = torch.empty(P, device=dev)
    if mode == "param":
        lo, hi = sharding.shard_range(P, 0, 1, sharding.ALIGN)
        sharding.param_sharded(Xd[:, lo:hi], w32, W, out[lo:hi])
    elif mode == "chain":
        sharding.client_sharded_chain(Xd, w32, W, out, n_blocks=5)
    else:
        sharding.client_sharded_allreduce(Xd, w32, W, out)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(exp))
