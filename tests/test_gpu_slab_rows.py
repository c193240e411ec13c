"""Client vectors written straight into the round's HBM slab
(fedsim_amd/utils/slab_rows.py, fedagg_pack_segments_f32): the layout of the
packed row is the reference's parameters_to_vector (fedsim/utils/
convert_parameters.py:78-94) bit for bit; rows reserved by the round
aggregator and committed by ``add`` reduce to the oracle's average; a
SlabRow behaves as an ordinary tensor everywhere else, keeps its value when
its row is reused or its slab released, and the round loop with real local
SGD on the GPU gives the same bits with and without slab rows."""
import random
from functools import partial

import numpy as np
import pytest
import torch
from torch import nn
from torch.nn.utils import parameters_to_vector

from conftest import bits
from oracle import ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


class Odd(nn.Module):
    """Parameters of ragged sizes (1, 3, 7, 77 ...) in separate allocations,
    plus one view into a shared buffer, so the segment table has unaligned
    boundaries and unaligned 16-B groups."""

    def __init__(self, scale=1):
        super().__init__()
        self.a = nn.Linear(13 * scale, 7)
        self.b = nn.Parameter(torch.randn(1))
        self.c = nn.Linear(7, 3 * scale + 2)
        self.d = nn.Parameter(torch.randn(77, 5))


def _agg(**kw):
    from fedsim_amd.utils import SerialAggregator

    return SerialAggregator(**kw)


@pytest.mark.parametrize("scale", [1, 64, 3000])
def test_pack_layout_is_parameters_to_vector(scale):
    from fedsim_amd.utils import vectorize_module

    torch.manual_seed(scale)
    m = Odd(scale).to(DEV)
    want = parameters_to_vector(m.parameters()).detach()
    P = want.numel()
    agg = _agg()
    row = agg.reserve("p", P, DEV)
    assert row is not None and row.in_slab
    got = vectorize_module(m, out=row)
    assert got is row
    np.testing.assert_array_equal(bits(row.materialize().cpu().numpy()), bits(want.cpu().numpy()))
    # one segment when the parameters are views of one vector, in order
    from fedsim_amd.utils import initialize_module
    from fedsim_amd import ops

    initialize_module(m, want + 1.0)
    _, nseg, _ = ops.segment_table([p.detach() for p in m.parameters()], DEV)
    assert nseg == 1
    row2 = agg.reserve("p", P, DEV)
    vectorize_module(m, out=row2)
    np.testing.assert_array_equal(bits(row2.materialize().cpu().numpy()),
                                  bits((want + 1.0).cpu().numpy()))


def test_reserved_rows_reduce_bitwise_with_other_sources():
    """Slab rows and borrowed HBM tensors interleaved (host tensors of the
    same clients into a host key alongside), a reservation that is never
    added (a diverged client), and a small ring that wraps: each average
    equals the oracle's over its added vectors.  A host vector added to the
    HIP key raises, as the reference's ``sum_v + new_v`` does."""
    from fedsim_amd.utils import vectorize_module

    K = 23
    models = []
    for k in range(K):
        torch.manual_seed(100 + k)
        models.append(Odd(40).to(DEV))
    vecs = [parameters_to_vector(m.parameters()).detach() for m in models]
    P = vecs[0].numel()
    w = [int(v) for v in np.random.default_rng(3).integers(50, 601, size=K)]
    for borrow, max_rows in ((True, 4096), (False, 3), (True, 2)):
        agg = _agg(borrow=borrow, max_rows=max_rows)
        added = []
        on_host = []
        kept = []
        for k in range(K):
            if k % 4 == 0:
                agg.reserve("p", P, DEV)  # reserved, then the client diverged
            if k % 3 == 0:
                agg.add("h", vecs[k].cpu(), w[k])
                on_host.append(k)
                if "p" in agg:
                    with pytest.raises(RuntimeError, match="same device"):
                        agg.add("p", vecs[k].cpu(), w[k])
                continue
            if k % 3 == 1:
                val = vecs[k].clone()
            else:
                val = vectorize_module(models[k], out=agg.reserve("p", P, DEV))
                if k % 2 == 0:
                    kept.append((val, vecs[k]))  # still alive when its row is reused
            agg.add("p", val, w[k])
            added.append(k)
            assert "p" in agg
        for key, rows in (("p", added), ("h", on_host)):
            out = agg.pop(key)
            assert out.device.type == ("cuda" if key == "p" else "cpu")
            X = np.stack([vecs[k].cpu().numpy() for k in rows])
            exp = ref.reduce(X, [w[k] for k in rows], W=sum(w[k] for k in rows))
            np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(exp))
        for row, v in kept:  # reused rows / released slab: the value is kept
            assert torch.equal(row.view(torch.int32), v.view(torch.int32))


def test_reservation_alone_creates_no_key():
    agg = _agg()
    assert agg.reserve("local_params", 1000, DEV) is not None
    assert "local_params" not in agg
    assert agg.pop_all() == {}


def test_slab_row_is_an_ordinary_tensor():
    from fedsim_amd.utils import vectorize_module

    torch.manual_seed(7)
    m = Odd(8).to(DEV)
    v = parameters_to_vector(m.parameters()).detach()
    row = vectorize_module(m, out=_agg().reserve("p", v.numel(), DEV))
    assert row.shape == v.shape and row.dtype == v.dtype and row.device == v.device
    assert torch.equal(row + 1, v + 1)
    assert torch.equal(row.clone(), v)
    assert torch.equal(row.cpu(), v.cpu())
    assert float(row.sum()) == float(v.sum())
    assert type(row * 2) is torch.Tensor


def test_pop_step_over_slab_rows_is_the_fused_slab_pass():
    """A round of slab rows ends in the fused blocked step (the bench's
    kernel) with the oracle's bits."""
    from fedsim_amd import ops
    from fedsim_amd.utils import vectorize_module

    K = 9
    models = []
    for k in range(K):
        torch.manual_seed(200 + k)
        models.append(Odd(500).to(DEV))
    vecs = [parameters_to_vector(m.parameters()).detach() for m in models]
    P = vecs[0].numel()
    w = [int(v) for v in np.random.default_rng(4).integers(50, 601, size=K)]
    agg = _agg(borrow=True, expected_rows=K)
    for k in range(K):
        agg.add("p", vectorize_module(models[k], out=agg.reserve("p", P, DEV)), w[k])
    entry = agg._members["p"]
    assert entry.n_pending == K and not entry.borrowed  # all K in the slab
    cloud0 = np.random.default_rng(5).normal(0, 0.05, size=P).astype(np.float32)
    cloud = torch.from_numpy(cloud0).to(DEV)
    agg.pop_step("p", ops.ServerStep("fedavg", cloud, lr=0.3))
    X = np.stack([v.cpu().numpy() for v in vecs])
    exp = ref.fedavg_sgd(ref.reduce(X, w, W=sum(w)), cloud0, 0.3)
    np.testing.assert_array_equal(bits(cloud.cpu().numpy()), bits(exp))


class _NoRows(object):
    """Aggregator factory without row reservation (the borrowed path)."""

    def __init__(self, **kw):
        from fedsim_amd.utils import SerialAggregator

        class Agg(SerialAggregator):
            def reserve(self, key, P, device):
                return None

        self.cls, self.kw = Agg, kw

    def __call__(self):
        return self.cls(**self.kw)


@pytest.mark.parametrize("rid", ["r5", "r8", "r9"])
def test_round_loop_local_sgd_same_bits_with_slab_rows(rid):
    """Real local SGD on the GPU (FedAvg / AdaBest / FedDyn clients): the
    round driver's default aggregator now takes the clients' vectors as slab
    rows; five rounds give the same bits as the borrowed-vector path."""
    import json
    import os

    from conftest import GOLDEN_DIR
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.utils import slab_rows
    from oracle import synthetic_fl as S

    with open(os.path.join(GOLDEN_DIR, "rounds.json")) as f:
        run = [r for r in json.load(f)["runs"] if r["id"] == rid][0]
    outs = []
    for factory in (None, _NoRows(borrow=True, expected_rows=5)):
        used = []
        orig = slab_rows.reserve_round_row

        def spy(key, module, _orig=orig, _used=used):
            row = _orig(key, module)
            _used.append(row is not None)
            return row

        import fedsim_amd.distributed.centralized.training.local_updates as LU
        LU.reserve_round_row = spy
        try:
            random.seed(S.RANDOM_SEED)
            torch.manual_seed(S.TORCH_SEED)
            alg = getattr(training, run["algorithm"])(
                data_manager=S.TensorDataManager(valid_size=run.get("valid_size", 0)),
                metric_logger=None, num_clients=S.NUM_CLIENTS, sample_scheme="uniform",
                sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
                criterion_def="CrossEntropyScore",
                optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device="cuda",
                aggregator_factory=factory, **run["alg_kwargs"])
            scores = alg.train(rounds=S.ROUNDS)
        finally:
            LU.reserve_round_row = orig
        assert all(used) == (factory is None) and used
        st = alg.get_server_storage()
        outs.append((st.read("cloud_params").detach().cpu().numpy(), scores))
    np.testing.assert_array_equal(bits(outs[0][0]), bits(outs[1][0]))
    assert outs[0][1] == outs[1][1]


@pytest.mark.parametrize("seed", range(16))
def test_pack_segments_random_layouts(seed):
    """Random parameter layouts: ragged sizes, views at unaligned offsets of
    one buffer (16-B and 4-B load paths, quads across segment boundaries),
    adjacent views that merge into one segment, every block width and row;
    the packed row reads back as torch.cat of the tensors, and no other row
    of the slab is touched."""
    from fedsim_amd import ops

    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 10))
    big = torch.randn(400_000, device=DEV)
    tensors, pos = [], int(rng.integers(0, 7))
    for i in range(n):
        size = int(rng.choice([1, 2, 3, 5, 4, 64, 1000, 4097, int(rng.integers(1, 60_000))]))
        if rng.random() < 0.5:  # a view of the shared buffer, maybe right after the last
            if rng.random() < 0.5:
                pos += int(rng.integers(0, 9))
            if pos + size > big.numel():
                pos = 0
            tensors.append(big[pos:pos + size])
            pos += size
        else:
            tensors.append(torch.randn(size, device=DEV))
    want = torch.cat(tensors)
    P = want.numel()
    C = int(rng.choice([1024, 2048, 4096]))
    Kcap = int(rng.integers(1, 5))
    r = int(rng.integers(0, Kcap))
    Xb = torch.full(ops.blocked_shape(Kcap, P, C), float("nan"), device=DEV)
    assert ops.pack_segments(tensors, Xb, r) == P
    got = ops.unpack_row(Xb, r, P)
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))
    others = [k for k in range(Kcap) if k != r]
    if others:
        assert torch.isnan(Xb[:, others, :]).all()


def test_slab_rows_carry_special_values_bitwise():
    """-0.0, subnormals, +-inf, NaN and huge values in the parameters go
    through the pack unchanged and reduce as the reference's arithmetic does
    (the oracle on the same vectors)."""
    from fedsim_amd.utils import vectorize_module

    specials = torch.tensor([-0.0, 0.0, 1e-45, -1e-40, 3e38, -3e38, float("inf"),
                             float("-inf"), float("nan"), 1.0, -2.5])
    K = 6
    models, vecs = [], []
    for k in range(K):
        torch.manual_seed(300 + k)
        m = Odd(30).to(DEV)
        with torch.no_grad():
            m.d.view(-1)[: specials.numel()] = specials.roll(k).to(DEV)
            m.a.weight.view(-1)[k] = -0.0
        models.append(m)
        vecs.append(parameters_to_vector(m.parameters()).detach().cpu().numpy())
    P = vecs[0].size
    w = [int(v) for v in np.random.default_rng(9).integers(50, 601, size=K)]
    agg = _agg(borrow=True)
    for k in range(K):
        agg.add("p", vectorize_module(models[k], out=agg.reserve("p", P, DEV)), w[k])
    out = agg.pop("p").cpu().numpy()
    exp = ref.reduce(np.stack(vecs), w, W=sum(w))
    nan = np.isnan(exp)
    assert nan.any() and np.array_equal(np.isnan(out), nan)  # NaN payloads may differ
    np.testing.assert_array_equal(bits(out[~nan]), bits(exp[~nan]))


def test_committed_row_cannot_be_written_again():
    """A reserved row is handed over by the reservation protocol: once added
    it belongs to the aggregator -- packing into it again raises, and torch
    ops on the SlabRow act on a private copy (the slab keeps the sum's bits)."""
    from fedsim_amd.utils import vectorize_module

    torch.manual_seed(3)
    m = torch.nn.Linear(40, 7).to(DEV)
    v = torch.nn.utils.parameters_to_vector(m.parameters()).detach().clone()
    agg = _agg(expected_rows=2)
    row = vectorize_module(m, out=agg.reserve("p", v.numel(), DEV))
    agg.add("p", row, 2)
    with pytest.raises(ValueError, match="already added"):
        vectorize_module(m, out=row)
    row.mul_(0)  # acts on the row's own copy, not on the slab
    assert torch.equal(agg.pop("p"), (0 + v * 2) / 2)
