"""The ABI's largest accepted P (2^30 columns: every per-row byte offset, and
a row's buffer-descriptor range, at the 32-bit limit) through each layout and
column mapping: sampled columns, including the last ones, against the oracle
bit for bit.  About 20 GB of HBM."""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref

pytestmark = pytest.mark.gpu

P = 1 << 30
K = 2


@pytest.fixture(scope="module")
def data():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fedsim_amd import ops

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2024)
    X = torch.empty((K, P), dtype=torch.float32, device=dev).uniform_(-1, 1, generator=g)
    w = [3, 7]
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    rng = np.random.default_rng(5)
    cols = np.unique(np.concatenate([rng.integers(0, P, 4096), np.arange(P - 4100, P),
                                     np.arange(0, 64)]))
    idx = torch.from_numpy(cols).to(dev)
    Xs = X[:, idx].cpu().numpy()
    want = ref.reduce(np.ascontiguousarray(Xs), w, W=sum(w))
    yield dict(dev=dev, X=X, w=w, w32=w32, idx=idx, want=want)
    del X
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mapping", ["auto", "wide", "narrow1", "narrow2", "narrow4"])
@pytest.mark.parametrize("layout", ["strided", "rows"])
def test_max_P(layout, mapping, data):
    from fedsim_amd import ops

    d = data
    out = torch.empty(P, dtype=torch.float32, device=d["dev"])
    fl = ops.tuning_flags(mapping=mapping)
    if layout == "strided":
        ops.reduce_slab(d["X"], d["w32"], out, W=sum(d["w"]), flags=fl)
    else:
        ops.reduce_rows([d["X"][0], d["X"][1]], d["w32"], out, W=sum(d["w"]), flags=fl)
    got = out[d["idx"]].cpu().numpy()
    np.testing.assert_array_equal(bits(got), bits(d["want"]))
    del out


def test_max_P_blocked_fused_step(data):
    """The column-blocked slab and the fused FedAvg step at P = 2^30."""
    from fedsim_amd import ops

    d = data
    Xb = ops.to_blocked(d["X"], 4096)
    cloud = torch.zeros(P, dtype=torch.float32, device=d["dev"])
    step = ops.ServerStep("fedavg", cloud, lr=1.0)
    ops.reduce_blocked_step(Xb, d["w32"], step, W=sum(d["w"]))
    del Xb
    got = cloud[d["idx"]].cpu().numpy()
    zero = np.zeros_like(d["want"])
    np.testing.assert_array_equal(bits(got), bits(ref.fedavg_sgd(d["want"], zero, 1.0)))
