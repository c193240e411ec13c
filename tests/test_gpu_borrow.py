"""Zero-copy rounds of HBM-resident client vectors (SerialAggregator(borrow=True),
fedagg_reduce_rows_f32 / fedagg_reduce_step_rows_f32): the client tensors are
reduced where they live, in arrival order, bit for bit equal to the oracle and
to the snapshotting path — across Bmax drains, interleaved with host adds,
with get() in the middle, and fused with every server step."""
import numpy as np
import pytest
import torch

from conftest import bits
from oracle import ref
from oracle import vectors as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


@pytest.mark.parametrize("P", [1, 3, 4, 1023, 65_537, 1_085_668])
@pytest.mark.parametrize("max_rows", [1, 3, 4096])
def test_borrowed_rows_bitwise(P, max_rows, dev):
    from fedsim_amd.utils import SerialAggregator

    K = 23
    X = V.client_rows("normal", K, P, 7)
    w = V.client_weights("fedavg", K, 7)
    agg = SerialAggregator(max_rows=max_rows, borrow=True)
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
    for k in range(K):
        agg.add("p", rows[k], w[k])
        if k == 11:
            mid = agg.get("p")
            np.testing.assert_array_equal(
                bits(mid.cpu().numpy()), bits(ref.reduce(X[:12], w[:12], W=sum(w[:12]))))
    assert len(agg._members["p"].borrowed) <= max(1, max_rows)
    out = agg.pop("p")
    assert out.device == dev
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.reduce(X, w, W=sum(w))))


def test_borrow_interleaved_with_host_and_unaligned_sources(dev):
    """Strided device views and misaligned device views (both snapshotted
    into the slab) between borrowed rows: arrival order is kept.  A host
    vector added to the HIP key raises as the reference's ``sum_v + new_v``
    does (aggregators.py:38,40) and leaves the rows as they were."""
    from fedsim_amd.utils import SerialAggregator

    K, P = 17, 10_007
    X = V.client_rows("realistic", K, P, 9)
    w = V.client_weights("fednova", K, 9)
    agg = SerialAggregator(borrow=True)
    big = torch.empty(P + 1, device=dev)
    wide = torch.empty(2 * P, device=dev)
    for k in range(K):
        if k == 5:
            with pytest.raises(RuntimeError, match="same device"):
                agg.add("p", torch.from_numpy(X[k].copy()), w[k])
        if k % 4 == 1:
            wide[::2].copy_(torch.from_numpy(X[k]))            # strided view: slab path
            src = wide[::2]
        elif k % 4 == 3:
            big[1:].copy_(torch.from_numpy(X[k]))              # 4-B offset view: slab path
            src = big[1:]
        else:
            src = torch.from_numpy(X[k].copy()).to(dev)        # borrowed
        agg.add("p", src, w[k])
        if k % 4 == 3:
            big.fill_(float("nan"))  # the misaligned view was snapshotted at add
        if k % 4 == 1:
            wide.fill_(float("nan"))  # so was the strided one
    out = agg.pop("p")
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.reduce(X, w, W=sum(w))))


def test_borrowed_tensor_mutated_in_place_raises(dev):
    from fedsim_amd.utils import SerialAggregator

    agg = SerialAggregator(borrow=True)
    t = torch.ones(4096, device=dev)
    agg.add("p", t, 1)
    t.mul_(2)
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.pop("p")
    # the snapshotting aggregator keeps the reference semantics instead
    agg2 = SerialAggregator(borrow=False)
    t = torch.ones(4096, device=dev)
    agg2.add("p", t, 1)
    t.mul_(2)
    assert torch.equal(agg2.pop("p"), torch.ones(4096, device=dev))


def test_borrowed_rows_on_another_stream(dev):
    """Client tensors produced on a side stream: reading them on the compute
    stream after the producer's work is ordered by the caller, and their
    memory is not reused before the reduction ran (record_stream)."""
    from fedsim_amd.utils import SerialAggregator

    K, P = 6, 300_001
    X = V.client_rows("normal", K, P, 2)
    w = [1] * K
    side = torch.cuda.Stream(dev)
    agg = SerialAggregator(borrow=True)
    for k in range(K):
        with torch.cuda.stream(side):
            t = torch.from_numpy(X[k].copy()).to(dev, non_blocking=False)
        torch.cuda.current_stream(dev).wait_stream(side)
        agg.add("p", t, w[k])
        del t
    out = agg.pop("p")
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.reduce(X, w, W=K)))


@pytest.mark.parametrize("algo", ["fedavg", "adabest", "feddyn"])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("P", [70_001, 70_002])
def test_borrowed_pop_step_matches_two_step(algo, momentum, P, dev):
    """pop_step over borrowed rows (one fedagg_reduce_step_rows_f32 launch)
    == pop + fedagg_server_step_f32, bitwise, for every algorithm epilogue.
    Odd P runs one column per lane; even P two (the early-operand code)."""
    from fedsim_amd import ops
    from fedsim_amd.utils import SerialAggregator

    K = 9
    X = V.client_rows("realistic", K, P, 4)
    w = V.client_weights("fedavg", K, 4)
    cloud0 = torch.from_numpy(V.cloud_vector(P, 5)).to(dev)
    aux0 = torch.from_numpy(V.cloud_vector(P, 6)).to(dev)
    outs = []
    for fused in (True, False):
        agg = SerialAggregator(borrow=True)
        for k in range(K):
            agg.add("p", torch.from_numpy(X[k].copy()).to(dev), w[k])
        cloud, aux = cloud0.clone(), aux0.clone()
        buf = torch.empty_like(cloud) if momentum else None
        grad = torch.empty_like(cloud)
        step = ops.ServerStep(algo, cloud, lr=0.3, momentum=momentum, coef=0.6,
                              aux=None if algo == "fedavg" else aux, momentum_buf=buf,
                              momentum_init=True, grad_out=grad)
        if fused:
            agg.pop_step("p", step)
        else:
            step.apply(agg.pop("p").reshape(-1))
        outs.append([t.cpu().numpy() for t in (cloud, aux, grad)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(bits(a), bits(b))
    avg = ref.reduce(X, w, W=sum(w))
    if algo == "fedavg" and not momentum:
        np.testing.assert_array_equal(bits(outs[0][0]),
                                      bits(ref.fedavg_sgd(avg, cloud0.cpu().numpy(), 0.3)))


def test_borrowed_full_size_round(dev):
    """Headline size through the borrowing aggregator: 1000 separate HBM
    client tensors of 25 M floats (100 GB).  The default HBM budget makes the
    aggregator drain once in the middle (accumulator chaining) and run the
    FedAvg step after the last drain (split, ops.fuse_step_pays); the result
    equals one fused pass of the row-pointer kernel bitwise, and the oracle on
    4096 sampled columns."""
    from fedsim_amd import ops
    from fedsim_amd.utils import SerialAggregator

    K, P = 1000, 25_000_000
    torch.cuda.empty_cache()  # earlier tests' cached blocks count as used
    free, _ = torch.cuda.mem_get_info(dev)
    if free < 130e9:
        pytest.skip("needs >130 GB of free HBM")
    g = torch.Generator(device=dev).manual_seed(8)
    rows = [torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g) for _ in range(K)]
    w = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    W = sum(w)
    agg = SerialAggregator(borrow=True)
    entry = None
    drains = 0
    for k in range(K):
        agg.add("p", rows[k], w[k])
        entry = agg._members["p"]
        drains += entry.acc is not None and len(entry.borrowed) == 1 and k > 0
    assert entry.Bmax < K and drains >= 1  # at least one chained drain happened
    cloud = torch.zeros(P, device=dev)
    step = ops.ServerStep("fedavg", cloud, lr=1.0)
    agg.pop_step("p", step)
    # one pass over the same rows, then the same step on the stored average
    avg = torch.empty(P, device=dev)
    w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
    ops.reduce_rows(rows, w32, avg, W=W, flags=ops.FEDAGG_NT)
    cloud2 = torch.zeros(P, device=dev)
    ops.ServerStep("fedavg", cloud2, lr=1.0).apply(avg)
    assert torch.equal(cloud.view(torch.int32), cloud2.view(torch.int32))
    cols = torch.from_numpy(np.random.default_rng(3).choice(P, size=4096, replace=False)).to(dev)
    sub = torch.stack([r.index_select(0, cols) for r in rows]).cpu().numpy()
    exp_avg = ref.reduce(sub, w, W=W)
    np.testing.assert_array_equal(bits(avg.index_select(0, cols).cpu().numpy()), bits(exp_avg))
    exp_cloud = ref.fedavg_sgd(exp_avg, np.zeros(4096, np.float32), 1.0)
    np.testing.assert_array_equal(bits(cloud.index_select(0, cols).cpu().numpy()), bits(exp_cloud))


@pytest.mark.parametrize("P", [5, 70_001, 70_002, 70_004])
@pytest.mark.parametrize("mapping", ["wide", "narrow1", "narrow2", "narrow4"])
@pytest.mark.parametrize("algo", ["fedavg", "adabest", "feddyn"])
def test_rows_step_mappings_bitwise(algo, mapping, P, dev):
    """fedagg_reduce_step_rows_f32 under each column mapping (two columns per
    lane falls back to one for odd P) == the oracle's reduce + server step."""
    from fedsim_amd import ops

    K = 11
    X = V.client_rows("realistic", K, P, 8)
    w = V.client_weights("fedavg", K, 8)
    W = sum(w)
    avg = ref.reduce(X, w, W=W)
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
    w32 = torch.tensor([ops.fl32(v) for v in w], dtype=torch.float32, device=dev)
    cloud0 = V.cloud_vector(P, 9)
    aux0 = V.cloud_vector(P, 10)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    aux = torch.from_numpy(aux0.copy()).to(dev)
    step = ops.ServerStep(algo, cloud, lr=0.3, coef=0.6,
                          aux=None if algo == "fedavg" else aux)
    ops.reduce_rows_step(rows, w32, step, W=W, mapping=mapping)
    want = ref.ServerState(algo, cloud0, dict(lr=0.3), coef=0.6,
                           aux=None if algo == "fedavg" else aux0)
    want.step(avg)
    np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(want.cloud))
    if algo != "fedavg":
        np.testing.assert_array_equal(bits(aux.cpu().numpy()), bits(want.aux))


@pytest.mark.parametrize("borrow", [True, False])
@pytest.mark.parametrize("algo", ["fedavg", "adabest"])
def test_pop_step_split_policy_bitwise(borrow, algo, dev):
    """At P in [2^20, 2^24) with >= 128 rows, pop_step stores the average and
    runs fedagg_server_step_f32 after it (ops.fuse_step_pays): the result is
    bit for bit the fused pass's, forced here through the library entry, and
    the oracle's for plain FedAvg SGD."""
    from fedsim_amd import ops
    from fedsim_amd.utils import SerialAggregator

    K, P = 130, (1 << 20) + 6
    assert not ops.fuse_step_pays(P, K)
    X = V.client_rows("realistic", K, P, 12)
    w = V.client_weights("fedavg", K, 12)
    cloud0 = torch.from_numpy(V.cloud_vector(P, 13)).to(dev)
    aux0 = torch.from_numpy(V.cloud_vector(P, 14)).to(dev)
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
    outs = []
    for via in ("aggregator", "fused_entry"):
        cloud, aux, grad = cloud0.clone(), aux0.clone(), torch.empty_like(cloud0)
        avg_out = torch.full_like(cloud0, float("nan"))
        step = ops.ServerStep(algo, cloud, lr=0.3, coef=0.6,
                              aux=None if algo == "fedavg" else aux, grad_out=grad,
                              avg_out=avg_out)
        if via == "aggregator":
            agg = SerialAggregator(borrow=borrow)
            for k in range(K):
                agg.add("p", rows[k], w[k])
            agg.pop_step("p", step)
        else:
            w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
            ops.reduce_rows_step(rows, w32, step, W=sum(w))
        outs.append([t.cpu().numpy() for t in (cloud, aux, grad, avg_out)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(bits(a), bits(b))
    avg = ref.reduce(X, w, W=sum(w))
    # avg_out is written on the split path too (ServerStep.apply copies it)
    np.testing.assert_array_equal(bits(outs[0][3]), bits(avg))
    if algo == "fedavg":
        np.testing.assert_array_equal(bits(outs[0][0]),
                                      bits(ref.fedavg_sgd(avg, cloud0.cpu().numpy(), 0.3)))


@pytest.mark.parametrize("K", [3, 21])
@pytest.mark.parametrize("P", [(1 << 22) + 130, (1 << 22) + 256 + 2, 1 << 22])
def test_borrowed_rows_two_pieces_bitwise(K, P, dev):
    """From P = 2^22 on, borrowed rows take the two-pieces-per-lane kernel (a
    wave reads 1 KiB of each row per visit): ragged last wave (second piece
    past P, or both pieces partial), fewer rows than one unrolled batch, and a
    batch tail. Plain reduce and fused FedAvg step vs the oracle, bitwise."""
    from fedsim_amd import ops

    X = V.client_rows("normal", K, P, 31)
    w = V.client_weights("fedavg", K, 31)
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
    w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
    out = torch.full((P,), float("nan"), device=dev)
    ops.reduce_rows(rows, w32, out, W=sum(w))
    avg = ref.reduce(X, w, W=sum(w))
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(avg))
    cloud0 = V.cloud_vector(P, 32)
    cloud = torch.from_numpy(cloud0.copy()).to(dev)
    grad = torch.empty_like(cloud)
    ops.reduce_rows_step(rows, w32, ops.ServerStep("fedavg", cloud, lr=0.3, grad_out=grad),
                         W=sum(w))
    np.testing.assert_array_equal(bits(cloud.cpu().numpy()),
                                  bits(ref.fedavg_sgd(avg, cloud0, 0.3)))


@pytest.mark.parametrize("init", [True, False])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("algo", ["adabest", "feddyn"])
def test_borrowed_rows_two_pieces_step_algos(algo, momentum, init, dev):
    """The two-piece kernel with the step operands read early and pinned
    (three per piece for AdaBest / FedDyn with momentum): fused step vs the
    oracle's server step, bitwise, with a fresh and a carried momentum
    buffer, at a P with a ragged two-piece tail."""
    from fedsim_amd import ops

    K, P = 21, (1 << 22) + 130
    X = V.client_rows("realistic", K, P, 33)
    w = V.client_weights("fedavg", K, 33)
    rows = [torch.from_numpy(X[k].copy()).to(dev) for k in range(K)]
    w32 = torch.tensor([ops.fl32(v) for v in w], device=dev)
    cloud0, aux0 = V.cloud_vector(P, 34), V.cloud_vector(P, 35)
    opt = dict(lr=0.3, momentum=momentum)
    st = ref.ServerState(algo, cloud0, opt, aux=aux0, coef=0.6)
    buf0 = None
    if momentum and not init:  # carry a buffer from a first oracle step
        st.step(V.cloud_vector(P, 36))
        buf0 = st.buf.copy()
    cloud_in = st.cloud.copy()
    aux_in = st.aux.copy()
    avg = ref.reduce(X, w, W=sum(w))
    st.step(avg)
    cloud = torch.from_numpy(cloud_in).to(dev)
    aux = torch.from_numpy(aux_in).to(dev)
    grad = torch.empty_like(cloud)
    buf = None
    if momentum:
        buf = torch.from_numpy(buf0).to(dev) if buf0 is not None else torch.empty_like(cloud)
    avg_prev = torch.empty_like(cloud) if algo == "feddyn" else None
    step = ops.ServerStep(algo, cloud, lr=0.3, momentum=momentum, coef=0.6, aux=aux,
                          avg_prev=avg_prev, momentum_buf=buf, momentum_init=buf0 is None,
                          grad_out=grad)
    ops.reduce_rows_step(rows, w32, step, W=sum(w))
    np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(st.cloud))
    np.testing.assert_array_equal(bits(aux.cpu().numpy()), bits(st.aux))
    np.testing.assert_array_equal(bits(grad.cpu().numpy()), bits(st.grad))
    if momentum:
        np.testing.assert_array_equal(bits(buf.cpu().numpy()), bits(st.buf))
    if algo == "feddyn":
        np.testing.assert_array_equal(bits(avg_prev.cpu().numpy()), bits(st.avg_prev))


_REUSED = {}


def _reuse_buffer_send(*args, **kwargs):
    """A client that writes every update into ONE persistent device buffer
    and returns that buffer (legal under the reference, which clones each
    message at training/utils.py:34)."""
    from oracle import synthetic_fl as S

    msg = S.synthetic_send_to_server(*args, **kwargs)
    v = msg["local_params"]
    buf = _REUSED.get(v.device)
    if buf is None:
        buf = _REUSED[v.device] = torch.empty_like(v)
    buf.copy_(v)
    msg["local_params"] = buf
    return msg


def test_client_reusing_its_buffer_matches_reference(dev):
    """The round driver's aggregator borrows HBM vectors; serial_aggregation
    must clone a vector whose ownership it cannot show, so a buffer-reusing
    client gets the reference's 5-round FedAvg trajectory bit for bit (no
    error, no stale rows), while a fresh vector is still borrowed."""
    import json
    import os
    import random
    from functools import partial

    from conftest import GOLDEN_DIR
    from fedsim_amd.distributed.centralized.training import FedAvg
    from oracle import synthetic_fl as S

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        run = [r for r in json.load(f)["runs"] if r["id"] == "r0"][0]
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        want = z["r0/cloud"]

    class Reusing(S.make_algorithm(FedAvg)):
        send_to_server = _reuse_buffer_send

    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = Reusing(data_manager=S.FakeDataManager(), metric_logger=None,
                  num_clients=S.NUM_CLIENTS, sample_scheme="uniform", sample_rate=S.SAMPLE_RATE,
                  model_def=S.TinyModel, epochs=1, criterion_def="CrossEntropyScore",
                  optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device="cuda")
    scores = alg.train(rounds=S.ROUNDS)
    got = alg.get_server_storage().read("cloud_params").detach().cpu().numpy()
    np.testing.assert_array_equal(bits(got), bits(want))
    assert {k: float(v) for k, v in scores.items()} == run["scores"]

    # outside the driver: a vector declared in the caller's own hand-over
    # round is borrowed (no copy); an undeclared one -- even one only its
    # message references -- and a kept one are cloned
    from fedsim_amd.distributed.centralized.training import serial_aggregation
    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.handover import hand_over, handover_round

    agg = SerialAggregator(borrow=True)
    with handover_round():
        msg = dict(local_params=hand_over(torch.ones(4096, device=dev)),
                   num_samples=dict(train=3), diverged=False, metrics=dict())
        ptr = msg["local_params"].data_ptr()
        assert serial_aggregation(None, 0, msg, "train", agg)
    entry = agg._members["local_params"]
    assert entry.borrowed[0][0].data_ptr() == ptr
    msg = dict(local_params=torch.ones(4096, device=dev), num_samples=dict(train=3),
               diverged=False, metrics=dict())
    ptr = msg["local_params"].data_ptr()
    assert serial_aggregation(None, 1, msg, "train", agg)
    assert entry.borrowed[1][0].data_ptr() != ptr
    kept = torch.ones(4096, device=dev)
    msg = dict(local_params=kept, num_samples=dict(train=3), diverged=False, metrics=dict())
    assert serial_aggregation(None, 2, msg, "train", agg)
    assert entry.borrowed[2][0].data_ptr() != kept.data_ptr()
    kept.fill_(5.0)  # the caller still owns it and may change it
    assert torch.equal(agg.pop("local_params"), torch.ones(4096, device=dev))


_KEPT_VIEWS = []


def _keep_view_send(id, rounds, storage, *a, **k):
    """A client that hands its fresh vector over but keeps a view of it; the
    NEXT client then writes through the previous client's view -- after that
    vector was received, before the round is reduced."""
    from oracle import synthetic_fl as S

    msg = S.synthetic_send_to_server(id, rounds, storage, *a, **k)
    for v in _KEPT_VIEWS:
        v.fill_(float("nan"))
    _KEPT_VIEWS.clear()
    _KEPT_VIEWS.append(msg["local_params"][:16])
    return msg


@pytest.mark.parametrize("keep_view", [False, True])
def test_driver_borrows_by_hand_over_token(keep_view, dev, monkeypatch):
    """Inside the round driver ownership is the client's explicit hand-over
    (utils/handover.py), not a reference count: the synthetic clients hand
    their fresh vectors over and every one is borrowed; a client that keeps a
    view of its output gets the reference's clone (the view is seen on the
    storage), so writes through the view after receive_from_client change
    nothing -- the 5-round trajectory is the reference's, bit for bit."""
    import json
    import os
    import random
    from functools import partial

    from conftest import GOLDEN_DIR
    from fedsim_amd.distributed.centralized.training import FedAvg
    from fedsim_amd.distributed.centralized.training import utils as U
    from oracle import synthetic_fl as S

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        run = [r for r in json.load(f)["runs"] if r["id"] == "r0"][0]
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        want = z["r0/cloud"]
    decisions = []
    real = U._handed_over
    monkeypatch.setattr(U, "_handed_over", lambda t: decisions.append(real(t)) or decisions[-1])
    base = S.make_algorithm(FedAvg)
    cls = type("KeepView", (base,), {"send_to_server": staticmethod(_keep_view_send)}) \
        if keep_view else base
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
              sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel,
              epochs=1, criterion_def="CrossEntropyScore",
              optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device="cuda")
    scores = alg.train(rounds=S.ROUNDS)
    _KEPT_VIEWS.clear()
    got = alg.get_server_storage().read("cloud_params").detach().cpu().numpy()
    np.testing.assert_array_equal(bits(got), bits(want))
    assert {k: float(v) for k, v in scores.items()} == run["scores"]
    assert len(decisions) == 25
    assert all(decisions) if not keep_view else not any(decisions)


@pytest.mark.parametrize("mode", ["auto", "zero_copy", "dma", "mixed"])
@pytest.mark.parametrize("borrow_host", [False, True])
def test_host_pack_modes_are_exact(dev, mode, borrow_host, monkeypatch):
    """Host vectors reach their slab rows either through the pack kernel
    reading the page-locked slot (or the caller's pinned tensor) in place over
    PCIe, or through a DMA into a device slot (aggregators._HOST_PACK): every
    mode gives the oracle's round bit for bit -- pageable and pinned sources,
    a pinned source at an offset that is not 16-byte aligned (the 2-D DMA),
    tails that are not a multiple of 4, and more rows than staging slots."""
    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils import aggregators as A

    monkeypatch.setattr(A, "_HOST_PACK", mode)
    for K, P in ((7, 4099), (5, 199_210), (4, A._ASYNC_STAGE_MIN + 5)):
        X = V.client_rows("realistic", K, P, 12)
        w = V.client_weights("fedavg", K, 12)
        agg = SerialAggregator(borrow=True, borrow_host=borrow_host, max_rows=3)
        pin_base = torch.empty(P + 1).pin_memory()
        for k in range(K):
            src = torch.from_numpy(X[k].copy())
            if k % 3 == 1:
                src = src.pin_memory()
            elif k % 3 == 2:  # pinned, 4 bytes off a 16-byte boundary
                src = pin_base[1:]
                src.copy_(torch.from_numpy(X[k]))
            agg.add("p", src, w[k])
            if k % 3 == 2:
                agg.get_sum("p")  # the shared pinned buffer is read before reuse
        np.testing.assert_array_equal(bits(agg.pop("p").numpy()),
                                      bits(ref.reduce(X, w, W=sum(w))))


@pytest.mark.parametrize("borrow_host", [False, True])
def test_split_staging_copy_keeps_the_tail(dev, borrow_host):
    """From 32 MB the staging copy runs on six memmove threads; at P = 6144m + 1
    floats the byte count is not a multiple of six pages' worth, and the
    last chunk must still reach the slot (every column bitwise, the last
    included)."""
    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _STAGE_SPLIT_MIN

    P = 6144 * 1366 + 1
    assert 4 * P >= _STAGE_SPLIT_MIN
    K = 3
    X = V.client_rows("realistic", K, P, 14)
    w = V.client_weights("fedavg", K, 14)
    agg = SerialAggregator(borrow=True, borrow_host=borrow_host)
    for k in range(K):
        agg.add("p", torch.from_numpy(X[k].copy()), w[k])
    out = agg.pop("p").numpy()
    np.testing.assert_array_equal(bits(out), bits(ref.reduce(X, w, W=sum(w))))


def test_handed_over_large_pinned_rows_are_checked_at_the_reduction(dev):
    """From 32 MB a handed-over pinned vector is DMA'd straight from the
    caller's buffer and the ingest worker does not wait for the DMA: the
    reduction does, and checks the vector's version there -- unchanged rows
    reduce bit for bit, a row changed in place before the round is reduced
    (even after its DMA completed) raises, as for a borrowed HBM row."""
    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _PINNED_DIRECT_MIN

    P = _PINNED_DIRECT_MIN // 4 + 5
    K = 3
    X = V.client_rows("realistic", K, P, 15)
    w = V.client_weights("fedavg", K, 15)
    rows = [torch.from_numpy(X[k].copy()).pin_memory() for k in range(K)]
    agg = SerialAggregator(borrow=True, borrow_host=True)
    for k in range(K):
        agg.add("p", rows[k], w[k])
    np.testing.assert_array_equal(bits(agg.pop("p").numpy()), bits(ref.reduce(X, w, W=sum(w))))
    agg = SerialAggregator(borrow=True, borrow_host=True)
    for k in range(K):
        agg.add("p", rows[k], w[k])
    torch.cuda.synchronize()  # every DMA has completed
    rows[1].mul_(2)
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.pop("p")


def test_handed_over_host_rows_are_staged_after_add(dev):
    """borrow_host=True with host vectors (the round driver's aggregator under
    device="cpu"): each handed-over vector is copied into pinned staging and
    DMA'd by the ingest worker after add returns (while the next client
    trains), in arrival order, interleaved with the HBM rows of another key
    (borrowed); both rounds are the oracle's bit for bit.  An HBM vector
    added to the host key raises (the reference's ``sum_v + new_v``)."""
    from fedsim_amd.utils import SerialAggregator

    K, P = 23, 600_001  # above _ASYNC_STAGE_MIN: the worker stages them
    X = V.client_rows("realistic", K, P, 8)
    w = V.client_weights("fedavg", K, 8)
    agg = SerialAggregator(borrow=True, borrow_host=True, max_rows=5)
    sel = [k for k in range(K) if k % 5 == 4]
    for k in range(K):
        src = torch.from_numpy(X[k].copy())
        agg.add("p", src, w[k])
        del src
        if k in sel:
            agg.add("d", torch.from_numpy(X[k].copy()).to(dev), w[k])
        if k == 9:
            with pytest.raises(RuntimeError, match="same device"):
                agg.add("p", torch.from_numpy(X[k].copy()).to(dev), w[k])
    out = agg.pop("p")
    assert out.device.type == "cpu"
    np.testing.assert_array_equal(bits(out.numpy()), bits(ref.reduce(X, w, W=sum(w))))
    ws = [w[k] for k in sel]
    outd = agg.pop("d")
    assert outd.device == dev
    np.testing.assert_array_equal(bits(outd.cpu().numpy()), bits(ref.reduce(X[sel], ws, W=sum(ws))))


def test_small_handed_over_host_rows_are_staged_at_add(dev):
    """Below _ASYNC_STAGE_MIN a handed-over host vector is staged on the
    calling thread at add (no worker hand-off), mixed with worker-staged
    large ones of another key; both rounds are the oracle's bit for bit."""
    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _ASYNC_STAGE_MIN

    K, Ps, Pl = 9, 199_210, _ASYNC_STAGE_MIN + 3
    Xs, Xl = V.client_rows("realistic", K, Ps, 10), V.client_rows("realistic", K, Pl, 11)
    w = V.client_weights("fedavg", K, 10)
    agg = SerialAggregator(borrow=True, borrow_host=True, max_rows=4)
    for k in range(K):
        agg.add("s", torch.from_numpy(Xs[k].copy()), w[k])
        agg.add("l", torch.from_numpy(Xl[k].copy()), w[k])
    np.testing.assert_array_equal(bits(agg.pop("s").numpy()), bits(ref.reduce(Xs, w, W=sum(w))))
    np.testing.assert_array_equal(bits(agg.pop("l").numpy()), bits(ref.reduce(Xl, w, W=sum(w))))


def test_release_after_failed_put_keeps_the_first_error(dev):
    """An entry whose staging put failed (a handed-over host vector changed
    before the worker copied it) can still be released: release() drains the
    copy stream and frees the slab without raising again (advisor, round 5),
    and the key's own reads keep raising the first error."""
    import threading

    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _ingest_for

    agg = SerialAggregator(borrow=True, borrow_host=True)
    gate = threading.Event()
    _ingest_for(dev).pool.submit(gate.wait)
    t = torch.ones(1 << 20)
    agg.add("p", t, 1)
    t.mul_(2)
    gate.set()
    e = agg._members["p"]
    with pytest.raises(RuntimeError, match="modified in place"):
        e._copies_issued()
    e.release()  # no second raise; the slab is dropped
    assert e.slab is None
    e.release()  # idempotent
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.get("p")
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.pop("p")


def test_handed_over_host_row_mutated_in_place_raises(dev):
    """A handed-over host vector changed in place before the ingest worker
    copied it is refused at the reduction (held back here so the change comes
    first: a change racing the copy itself is the caller's contract breach,
    as for borrowed HBM rows)."""
    import threading

    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _ingest_for

    agg = SerialAggregator(borrow=True, borrow_host=True)
    gate = threading.Event()
    _ingest_for(dev).pool.submit(gate.wait)  # the worker is busy until released
    t = torch.ones(1 << 20)
    agg.add("p", t, 1)
    t.mul_(2)
    gate.set()
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.pop("p")


@pytest.mark.parametrize("pinned", [False, True])
def test_earlier_handed_over_row_failure_is_not_lost(dev, pinned):
    """Two handed-over host rows staged by the worker; the FIRST is changed
    in place before its copy.  The later row's put succeeds, but the round
    must still refuse: every pending put is checked at the reduction, not
    only the newest (pageable sources: memmove into staging; pinned ones:
    DMA'd straight from the caller's buffer)."""
    import threading

    from fedsim_amd.utils import SerialAggregator
    from fedsim_amd.utils.aggregators import _ingest_for

    agg = SerialAggregator(borrow=True, borrow_host=True)
    gate = threading.Event()
    _ingest_for(dev).pool.submit(gate.wait)  # the worker is busy until released
    a, b = torch.ones(1 << 20), torch.full((1 << 20,), 2.0)
    if pinned:
        a, b = a.pin_memory(), b.pin_memory()
    agg.add("p", a, 1)
    agg.add("p", b, 1)
    a.mul_(3)
    gate.set()
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.get("p")
    with pytest.raises(RuntimeError, match="modified in place"):
        agg.pop("p")  # still refused: the ring lacks that row
    # the next round's aggregator is unaffected
    agg = SerialAggregator(borrow=True, borrow_host=True)
    agg.add("q", b, 1)
    assert torch.equal(agg.pop("q"), b)


def test_host_client_keeping_its_vector_is_cloned(dev):
    """serial_aggregation under the borrowing aggregator: a host vector the
    client still references is cloned (the reference's snapshot), so changing
    it after receive_from_client does not change the round."""
    from fedsim_amd.distributed.centralized.training.utils import serial_aggregation
    from fedsim_amd.utils import SerialAggregator, Storage

    K, P = 6, 65_537
    X = V.client_rows("realistic", K, P, 9)
    w = V.client_weights("fedavg", K, 9)
    agg = SerialAggregator(borrow=True, borrow_host=True)
    kept = []
    for k, msg in enumerate(V.client_messages(X, w)):
        kept.append(msg["local_params"])  # the client keeps its tensor
        assert serial_aggregation(Storage(), k, msg, "train", agg)
        kept[-1].fill_(float("nan"))
    out = agg.pop("local_params")
    np.testing.assert_array_equal(bits(out.numpy()), bits(ref.reduce(X, w, W=sum(w))))
