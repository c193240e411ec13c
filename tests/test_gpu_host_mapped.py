"""Page-locked host memory as kernel operands (fedagg_host_mapped, ABI 6):
the server step of FedSim's device="cpu" runs reads and writes the host
state in place over PCIe instead of copying it each way.

* ops.host_mapped: pinned host tensors (and views into them) are mapped at
  their own address; pageable, HBM and empty-pinned-slice cases as stated;
* a ServerStep whose operands are pinned host tensors and whose device is the
  GPU gives the oracle's step bit for bit -- fused into the last drain of a
  slab or of borrowed rows, and on a stored average -- for every algorithm x
  SGD configuration; a pageable operand is refused;
* the host-state step of the plugin surface (training/utils.py
  _fused_server_step_host) gives the same cloud, grad, momentum buffer and
  aux vectors in its zero-copy and DMA modes, round after round.
"""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu

OPTS = {
    "plain_lr0.3": dict(lr=0.3),
    "momentum_first": dict(lr=0.5, momentum=0.9),
    "momentum_damp_wd": dict(lr=0.1, momentum=0.8, dampening=0.25, weight_decay=1e-3),
    "nesterov": dict(lr=0.7, momentum=0.5, nesterov=True),
    "maximize_wd": dict(lr=1.0, weight_decay=0.01, maximize=True),
}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fedsim_amd import _native

    _native.load()
    return torch.device("cuda:0")


def test_host_mapped(dev):
    from fedsim_amd import ops

    pinned = torch.empty(10_001).pin_memory()
    assert ops.host_mapped(pinned)
    assert ops.host_mapped(pinned[3:77])  # a view inside the allocation
    assert ops.host_mapped(pinned[5:5])   # empty
    assert not ops.host_mapped(torch.empty(10_001))         # pageable
    assert not ops.host_mapped(torch.empty(64, device=dev))  # HBM
    assert not ops.host_mapped(np.zeros(4))


def _mapped_step(st, coef, algo, opt, dev, pad):
    """The step's operands as page-locked host tensors (rows of one padded
    buffer when ``pad``: 16-byte aligned, the fused entries' requirement)."""
    from fedsim_amd import ops

    P = st.cloud.size
    names = ["cloud", "grad"] + (["aux"] if st.aux is not None else []) + \
        (["buf"] if opt.get("momentum") else []) + (["avg_prev"] if algo == "feddyn" else [])
    pitch = -(-P // 4) * 4 if pad else P
    H = torch.empty(len(names) * pitch + (0 if pad else 1)).pin_memory()
    base = 0 if pad else 1  # unpadded: every row 4 bytes off a 16-byte boundary
    d = {n: H[base + i * pitch: base + i * pitch + P] for i, n in enumerate(names)}
    d["cloud"].copy_(torch.from_numpy(np.asarray(st.cloud, dtype=np.float32)))
    if "aux" in d:
        d["aux"].copy_(torch.from_numpy(np.asarray(st.aux, dtype=np.float32)))
    if "buf" in d and st.buf is not None:
        d["buf"].copy_(torch.from_numpy(np.asarray(st.buf, dtype=np.float32)))
    mom = opt.get("momentum", 0.0)
    step = ops.ServerStep(algo, d["cloud"], lr=opt["lr"], momentum=mom,
                          dampening=opt.get("dampening", 0.0),
                          weight_decay=opt.get("weight_decay", 0.0),
                          nesterov=opt.get("nesterov", False), maximize=opt.get("maximize", False),
                          coef=coef, aux=d.get("aux"), avg_prev=d.get("avg_prev"),
                          momentum_buf=d.get("buf"), momentum_init=(mom != 0 and st.buf is None),
                          grad_out=d["grad"], device=dev)
    return step, d


def _check(st, d, algo, opt):
    np.testing.assert_array_equal(bits(d["cloud"].numpy()), bits(st.cloud))
    np.testing.assert_array_equal(bits(d["grad"].numpy()), bits(st.grad))
    if st.aux is not None:
        np.testing.assert_array_equal(bits(d["aux"].numpy()), bits(st.aux))
    if opt.get("momentum"):
        np.testing.assert_array_equal(bits(d["buf"].numpy()), bits(st.buf))
    if algo == "feddyn":
        np.testing.assert_array_equal(bits(d["avg_prev"].numpy()), bits(st.avg_prev))


def _state(algo, o, P, seed, prebuf):
    aux = V.cloud_vector(P, seed + 2) if algo != "fedavg" else None
    coef = 0.6 if algo == "adabest" else (0.37 if algo == "feddyn" else 0.0)
    st = ref.ServerState(algo, V.cloud_vector(P, seed + 1), o, aux=aux, coef=coef)
    if prebuf and o.get("momentum"):
        st.buf = V.cloud_vector(P, seed + 4)
    return st, coef


@pytest.mark.parametrize("path", ["blocked_fused", "rows_fused", "apply", "apply_unaligned"])
@pytest.mark.parametrize("P", [5, 4099, 199_210])
@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("algo", ["fedavg", "adabest", "feddyn"])
def test_step_on_host_mapped_operands(algo, opt, P, path, dev):
    from fedsim_amd import ops

    o = OPTS[opt]
    K, seed = 9, 2000 + P % 89
    X = V.client_rows("realistic", K, P, seed)
    w = V.client_weights("fedavg", K, seed)
    W = sum(w)
    avg = ref.reduce(X, w, W=W)
    st, coef = _state(algo, o, P, seed, prebuf=(opt == "momentum_damp_wd"))
    step, d = _mapped_step(st, coef, algo, o, dev, pad=(path != "apply_unaligned"))
    st.step(avg)
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    if path == "blocked_fused":
        Xb = ops.to_blocked(torch.from_numpy(X).to(dev), ops.choose_block_cols(P))
        ops.reduce_blocked_step(Xb, w32, step, W=W)
    elif path == "rows_fused":
        rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
        ops.reduce_rows_step(rows, w32, step, W=W)
    else:
        step.apply(torch.from_numpy(np.asarray(avg, dtype=np.float32)).to(dev))
    torch.cuda.synchronize()
    _check(st, d, algo, o)


def test_pageable_operand_is_refused(dev):
    from fedsim_amd import ops

    cloud = torch.zeros(64).pin_memory()
    with pytest.raises(ValueError, match="the step runs on"):
        ops.ServerStep("fedavg", cloud, lr=1.0, grad_out=torch.zeros(64), device=dev)
    with pytest.raises(ValueError, match="the step runs on"):
        ops.ServerStep("fedavg", torch.zeros(64), lr=1.0, device=dev)


@pytest.mark.parametrize("pinned_cloud", [False, True])
@pytest.mark.parametrize("algo", ["FedAvg", "AdaBest", "FedDyn"])
@pytest.mark.parametrize("opt", ["plain", "momentum"])
def test_host_step_modes_agree(algo, opt, pinned_cloud, dev, monkeypatch):
    """Three rounds of the plugin surface with the cloud on the host: the
    zero-copy and DMA host steps leave the same state, bit for bit.  A
    page-locked cloud (what init_cloud makes) and its momentum buffer are
    stepped in place, as optimizer.step() updates them."""
    from fedsim_amd.distributed.centralized import training as T
    from fedsim_amd.distributed.centralized.training import utils as U
    from fedsim_amd.utils import SerialAggregator, Storage

    K, P = 6, 70_001
    kw = dict(lr=0.5, momentum=0.9) if opt == "momentum" else dict(lr=1.0)
    cls = getattr(T, algo)
    res = {}
    for mode in ("zero_copy", "dma"):
        monkeypatch.setattr(U, "_HOST_STEP", mode)
        torch.manual_seed(3)
        cloud = torch.randn(P)
        if pinned_cloud:
            cloud = cloud.pin_memory()
        cloud.requires_grad_()
        ptrs = set()
        st = Storage()
        st.write("cloud_params", cloud)
        st.write("optimizer", torch.optim.SGD(params=[cloud], **kw))
        st.write("lr_scheduler", None)
        st.write("avg_params", cloud.clone().detach())
        st.write("h", torch.zeros_like(cloud))
        st.write("beta", 0.6)
        st.write("num_clients", 20)
        stats = SerialAggregator()
        stats.add("avg_m", 0, 0)
        st.write("running_stats", stats)
        for rnd in range(3):
            X = V.client_rows("realistic", K, P, 40 + rnd)
            w = V.client_weights("fedavg", K, 40 + rnd)
            agg = SerialAggregator(expected_rows=K)
            for k, msg in enumerate(V.client_messages(X, w)):
                cls.receive_from_client(st, k, msg, "train", agg, None)
            cls.optimize(st, agg, None)
            buf = st.read("optimizer").state[cloud].get("momentum_buffer")
            ptrs.add((cloud.data_ptr(), None if buf is None or rnd == 0 else buf.data_ptr()))
        assert cloud.is_pinned() == pinned_cloud
        if pinned_cloud and mode == "zero_copy":
            assert len(ptrs) <= 2  # the same cloud and (from round 2 on) buffer storage
        state = [cloud.detach().clone(), cloud.grad.clone(), st.read("avg_params").clone(),
                 st.read("h").clone()]
        buf = st.read("optimizer").state[cloud].get("momentum_buffer")
        if buf is not None:
            state.append(buf.clone())
        res[mode] = state
    assert len(res["zero_copy"]) == len(res["dma"])
    for a, b in zip(res["zero_copy"], res["dma"]):
        assert a.device.type == "cpu" and torch.equal(a.view(torch.int32), b.view(torch.int32))
