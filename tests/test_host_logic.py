"""Host-side logic of the boundary, CPU only: scalar-key aggregation semantics,
serial_aggregation's call contract, Storage, AppendixAggregator, the server
optimizer detection of the fused step, and the round driver's plumbing."""
import random

import pytest
import torch

from conftest import golden_cases


class Recorder(object):
    """Aggregator stand-in recording serial_aggregation's add() calls."""

    def __init__(self):
        self.calls = []

    def add(self, key, value, weight=None):
        self.calls.append((key, value if not isinstance(value, torch.Tensor) else "T", weight))


def test_serial_aggregation_contract():
    from fedsim_amd.distributed.centralized.training import serial_aggregation

    msg = dict(local_params=torch.zeros(3), diverged=False, num_steps=2,
               num_samples={"train": 7, "test": 3},
               metrics={"train": {"loss": 1.5}, "test": {"acc": 0.5}})
    r = Recorder()
    assert serial_aggregation(None, 0, dict(msg), "train", r)
    # other_weight is sticky after the first split (reference quirk, utils.py:48-49)
    assert r.calls == [("local_params", "T", 7), ("clients.train.loss", 1.5, 7),
                       ("clients.test.acc", 0.5, 7)]
    r = Recorder()
    assert serial_aggregation(None, 0, dict(msg), "train", r, train_weight=1, other_weight=2)
    assert r.calls[0] == ("local_params", "T", 1) and r.calls[1][2] == 2
    r = Recorder()
    assert serial_aggregation(None, 0, dict(msg, num_samples={"train": 0, "test": 1}), "train",
                              r) is True
    assert r.calls == []  # weight <= 0: skipped (utils.py:45)
    r = Recorder()
    assert serial_aggregation(None, 0, dict(msg, diverged=True), "train", r) is False
    assert r.calls == []


def test_scalar_keys_match_reference_semantics():
    from fedsim_amd.utils import SerialAggregator

    a = SerialAggregator()
    a.add("x", 2, 3)
    a.add("x", 4.5, 1)
    assert a.get("x") == (0 + 2 * 3 + 4.5 * 1) / 4
    assert a.get_sum("x") == 10.5 and a.get_weight("x") == 4
    a.add("z", 1.0, 0)
    assert a.get("z") == 0  # zero weight -> raw sum (aggregators.py:56-57)
    t = torch.tensor(2.0)  # 0-dim tensors stay on the host path
    a.add("t", t, 2)
    assert float(a.pop("t")) == 2.0
    assert list(a.keys()) == ["x", "z"]
    assert dict(a.items()) == {"x": 10.5 / 4, "z": 0.0}
    assert a.pop_all() == {"x": 10.5 / 4, "z": 0.0}
    assert "x" not in a
    with pytest.raises(Exception, match="not in the aggregator"):
        a.get("x")
    with pytest.raises(TypeError):
        a.add("n", 1.0)  # weight=None -> 0 + None (aggregators.py:40)


def test_scalar_reports_match_golden():
    """Replaying the per-split metric adds of every golden case through the
    host path gives the reference's pop_all() reports exactly."""
    from fedsim_amd.utils import SerialAggregator
    from oracle import vectors as V

    n = 0
    for case in golden_cases():
        if "opts" in case or not all(case["ok"]) or case["reports"] is None:
            continue
        X = V.client_rows(case["dist"], case["K"], 1, case["seed"])  # P irrelevant here
        msgs = V.client_messages(X, case["weights"])
        a = SerialAggregator()
        for k, msg in enumerate(msgs):
            if case["algo"] in ("adabest", "feddyn"):
                tw = 1
            elif case["algo"] == "fednova":
                tw = case["weights"][k]
            else:
                tw = msg["num_samples"]["train"]
            if tw <= 0:
                continue
            other = None
            for split, ms in msg["metrics"].items():
                if other is None:
                    other = msg["num_samples"][split]
                for key, m in ms.items():
                    a.add(f"clients.{split}.{key}", m, other)
        assert {k: float(v) for k, v in a.pop_all().items()} == case["reports"], case["id"]
        n += 1
    assert n > 50


def test_storage_protection_semantics(capsys):
    from fedsim_amd.utils import Storage

    s = Storage()
    s.write("a", 1, read_protected=True, write_protected=True)
    assert s.read("a") == 1
    assert "read-protected" in capsys.readouterr().out
    assert s.read("a", silent=True) == 1
    s.write("a", 2)
    assert "over-written" in capsys.readouterr().out
    assert s.read("missing") is None
    assert s.get_protection_status("a") == (False, False)
    s.change_protection("a", True, False)
    assert "a" not in s.get_keys() and "a" in s.get_all_keys()
    s.remove("a")
    with pytest.raises(Exception):
        s.remove("a")


def test_appendix_aggregator():
    from fedsim_amd.utils import AppendixAggregator

    a = AppendixAggregator(max_deque_lenght=2)
    a.append("s", 1.0, weight=1, step=0)
    a.append("s", 2.0, weight=3, step=1)
    a.append("s", 4.0, weight=1, step=2)  # evicts the first entry
    assert a.get("s") == (2.0 * 3 + 4.0) / 4
    assert a.get("s", k=1) == 4.0
    # reference quirk (aggregators.py:211-215): k=0 slices [-0:], i.e. everything
    assert a.get("s", k=0) == a.get("s") == a.get("s", k=99)
    assert list(a.get_steps("s")) == [1, 2]
    assert not hasattr(a, "pop_step")
    with pytest.raises(Exception, match="is not in the aggregator"):
        a.get("missing")
    a.append_all({"t": 5.0}, step=3)
    assert a.pop_all() == {"s": (2.0 * 3 + 4.0) / 4, "t": 5.0}


def test_sgd_config_detection():
    from fedsim_amd.distributed.centralized.training.utils import plain_sgd_lr, sgd_config

    p = torch.zeros(10, requires_grad=True)
    assert plain_sgd_lr(torch.optim.SGD([p], lr=0.5), p) == 0.5
    cfg = sgd_config(torch.optim.SGD([p], lr=0.1, momentum=0.9, nesterov=True), p)
    assert cfg == dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0, nesterov=True,
                       maximize=False)
    assert plain_sgd_lr(torch.optim.SGD([p], lr=0.1, momentum=0.9), p) is None
    assert sgd_config(torch.optim.Adam([p], lr=0.1), p) is None
    q = torch.zeros(3, requires_grad=True)
    assert sgd_config(torch.optim.SGD([p, q], lr=0.1), p) is None
    assert sgd_config(torch.optim.SGD([q], lr=0.1), p) is None
    d = torch.zeros(4, dtype=torch.float64, requires_grad=True)
    assert sgd_config(torch.optim.SGD([d], lr=0.1), d) is None


def test_round_driver_plumbing_cpu():
    """The round loop with a recording aggregator (no GPU): rounds+1 rounds,
    client sampling, the static-method check, divergence early return."""
    from fedsim_amd.distributed.centralized import CentralFLAlgorithm
    from oracle import synthetic_fl as S

    seen = []

    class Agg(object):
        def __init__(self):
            self.n = 0

        def add(self, *a):
            self.n += 1

        def __contains__(self, k):
            return False

        def pop_all(self):
            return {}

    class Algo(CentralFLAlgorithm):
        def init(server_storage):
            server_storage.write("cloud_params", torch.zeros(3))

        def send_to_client(server_storage, client_id):
            return {}

        def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                           criterion, train_batch_size, inference_batch_size, optimizer_def,
                           lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
            seen.append((rounds, id))
            return dict(local_params=torch.zeros(3), num_steps=1, diverged=(id == 13),
                        num_samples={"train": 1}, metrics={})

        def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                                serial_aggregator, appendix_aggregator):
            return not client_msg["diverged"]

        def optimize(server_storage, serial_aggregator, appendix_aggregator):
            return {}

        def deploy(server_storage):
            return {}

        def report(server_storage, dataloaders, rounds, scores, metric_logger, device,
                   optimize_reports, deployment_points=None):
            return {"r": float(rounds)}

    random.seed(0)
    alg = Algo(data_manager=S.FakeDataManager(10), metric_logger=None, num_clients=10,
               sample_scheme="sequential", sample_rate=0.3, model_def=S.TinyModel, epochs=1,
               criterion_def="CrossEntropyScore", aggregator_factory=Agg)
    out = alg.train(rounds=2)
    assert [r for r, _ in seen] == [0, 0, 0, 1, 1, 1, 2, 2, 2]
    assert [c for _, c in seen] == [0, 1, 2, 3, 4, 5, 6, 7, 8]
    assert out == {"r": 1.0} and alg.get_round_number() == 3

    class Bad(Algo):
        def deploy(self, server_storage):
            return {}

    with pytest.raises(Exception, match="static"):
        Bad(data_manager=S.FakeDataManager(10), metric_logger=None, num_clients=10,
            sample_scheme="uniform", sample_rate=0.3, model_def=S.TinyModel, epochs=1,
            criterion_def="CrossEntropyScore", aggregator_factory=Agg)
    with pytest.raises(Exception, match="invalid client sample size"):
        Algo(data_manager=S.FakeDataManager(10), metric_logger=None, num_clients=10,
             sample_scheme="uniform", sample_rate=0.01, model_def=S.TinyModel, epochs=1,
             criterion_def="CrossEntropyScore")
    # divergence aborts training (centralized_fl_algorithm.py:427-432)
    seen.clear()
    alg2 = Algo(data_manager=S.FakeDataManager(20), metric_logger=None, num_clients=20,
                sample_scheme="sequential", sample_rate=0.5, model_def=S.TinyModel, epochs=1,
                criterion_def="CrossEntropyScore", aggregator_factory=Agg)
    alg2.train(rounds=3)
    assert seen[-1][1] == 13 and alg2.get_round_number() == 1


def test_pack_unpack_layout_and_views():
    """vectorize_module = concatenation of module.parameters() in registration
    order, each parameter's row-major storage (convert_parameters.py:78-94);
    initialize_module / vector_to_parameters hand out views of the (cloned)
    flat vector without further copies (convert_parameters.py:129-148)."""
    from fedsim_amd.utils.convert_parameters import (
        initialize_module, vector_to_named_parameters_like, vector_to_parameters_like,
        vectorize_module)

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                                torch.nn.Linear(4 * 6 * 6, 5))
    vec = vectorize_module(model)
    exp = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.equal(vec, exp) and not vec.requires_grad
    assert vec.numel() == sum(p.numel() for p in model.parameters())
    # unpack into a second model: same values, parameters are views of one buffer
    other = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                                torch.nn.Linear(4 * 6 * 6, 5))
    src = vec * 2
    assert initialize_module(other, src, clone=True)
    for p, q in zip(other.parameters(), model.parameters()):
        assert torch.equal(p.detach(), 2 * q.detach())
    ptrs = [p.data_ptr() for p in other.parameters()]
    base = next(other.parameters()).data_ptr()
    offs = [(q - base) // 4 for q in ptrs]
    assert offs == [0] + list(torch.cumsum(torch.tensor(
        [p.numel() for p in other.parameters()]), 0)[:-1].tolist())
    src.zero_()  # clone=True: the model does not alias the caller's vector
    assert torch.equal(next(other.parameters()).detach(), 2 * next(model.parameters()).detach())
    # size mismatch is reported, not raised (reference returns False)
    assert not initialize_module(other, vec[:-1])
    views = vector_to_parameters_like(vec, model.parameters())
    assert all(v.data_ptr() >= vec.data_ptr() for v in views)
    named = vector_to_named_parameters_like(vec, model.named_parameters())
    assert list(named) == [n for n, _ in model.named_parameters()]
    assert torch.equal(named["3.bias"], model[3].bias.detach())
    with pytest.raises(TypeError):
        vector_to_parameters_like([1.0], model.parameters())


def test_algorithm_registry_resolves_reference_names():
    """--algorithm <Name> resolution (fedsim_cli/utils.py:186-192): every
    reference class name maps to the plugin exported under that name."""
    from fedsim_amd.distributed import centralized
    from fedsim_amd.distributed.centralized import training

    for name in ("FedAvg", "AdaBest", "FedDyn", "FedNova", "FedProx", "FedDF"):
        cls = training.get_algorithm(name)
        assert cls is getattr(training, name) is getattr(centralized, name)
        assert cls.__name__ == name
    with pytest.raises(ValueError):
        training.get_algorithm("FedSGD")


def test_vectorize_module_grads_and_misc_helpers():
    """vectorize_module_grads (convert_parameters.py:97-126): None until every
    parameter has a gradient, then the gradients packed in parameter order;
    set_seed / get_from_module (random_utils.py, import_utils.py)."""
    import random

    import numpy as np
    import torch

    from fedsim_amd.utils import get_from_module, set_seed, vectorize_module_grads

    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Linear(4, 2))
    assert vectorize_module_grads(m) is None
    m(torch.randn(5, 3)).sum().backward()
    want = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    got = vectorize_module_grads(m)
    assert torch.equal(got, want) and got.data_ptr() != want.data_ptr()
    m[1].bias.grad = None
    assert vectorize_module_grads(m) is None

    set_seed(5, use_cuda=False)
    a = (np.random.rand(), random.random(), torch.rand(1).item())
    set_seed(5, use_cuda=False)
    assert a == (np.random.rand(), random.random(), torch.rand(1).item())

    assert get_from_module("fedsim_amd.utils", "Storage").__name__ == "Storage"
    assert get_from_module("fedsim_amd.utils", "nope") is None


def test_weight_rounding_matches_aten():
    """The aggregator's fl32(weight) (struct round trip) equals numpy's / ATen's
    round-to-nearest-even for the weight types serial_aggregation passes."""
    import numpy as np
    import torch

    from fedsim_amd.utils.aggregators import _fl32

    vals = [0, 1, 437, 2**24 + 1, 2**25 + 3, 0.1, 1 / 3, -2.5, 1e-45, 3.4e38, 5e-324,
            np.int64(600), np.float64(0.7), torch.tensor(123.456, dtype=torch.float64), True]
    for v in vals:
        assert _fl32(v) == float(np.float32(float(v))), v
        assert _fl32(v) == float(torch.tensor(float(v), dtype=torch.float32)), v


def test_feddf_target_reuse_conditions():
    """FedDF reuses a batch's ensemble targets across global epochs only for
    an in-order loader and a pure forward (no buffers, no train-mode dropout),
    where recomputing them, as the reference does, gives the same values."""
    import torch
    from torch import nn
    from torch.utils.data import DataLoader, TensorDataset

    from fedsim_amd.distributed.centralized.training.feddf import _in_order, _pure_forward

    ds = TensorDataset(torch.zeros(10, 2), torch.zeros(10))
    assert _in_order(DataLoader(ds, batch_size=4))
    assert not _in_order(DataLoader(ds, batch_size=4, shuffle=True))
    assert _pure_forward(nn.Sequential(nn.Linear(2, 3), nn.ReLU(), nn.Linear(3, 2)))
    assert not _pure_forward(nn.Sequential(nn.Linear(2, 3), nn.BatchNorm1d(3)))
    drop = nn.Sequential(nn.Linear(2, 3), nn.Dropout(0.5))
    assert not _pure_forward(drop)
    drop.eval()
    assert _pure_forward(drop)


def test_client_context_fingerprint():
    """The plain-data image of a send_to_client message that client-sharded
    rounds compare (centralized_fl_algorithm._context_fingerprint): exact
    floats (hex), small tensors by value, models and large tensors skipped."""
    import math

    import numpy as np
    import torch

    from fedsim_amd.distributed.centralized.centralized_fl_algorithm import (
        _context_fingerprint)

    model = torch.nn.Linear(3, 2)
    a = _context_fingerprint(dict(model=model, average_sample=0.1, mu=0.01, n=3,
                                  t=torch.tensor([1.0, 2.0]), big=torch.zeros(100),
                                  s="x", np=np.float32(0.5), none=None, tup=(1, 2.0)))
    assert set(a) == {"average_sample", "mu", "n", "t", "s", "np", "none", "tup"}
    b = _context_fingerprint(dict(model=torch.nn.Linear(3, 2), average_sample=0.1, mu=0.01,
                                  n=3, t=torch.tensor([1.0, 2.0]), big=torch.ones(100), s="x",
                                  np=np.float32(0.5), none=None, tup=(1, 2.0)))
    assert a == b  # models and big tensors do not take part
    c = _context_fingerprint(dict(average_sample=math.nextafter(0.1, 1.0)))
    assert c["average_sample"] != a["average_sample"]  # one ulp is a difference
    assert _context_fingerprint(dict(x=float("nan"))) == _context_fingerprint(dict(x=float("nan")))
    assert _context_fingerprint(None) is None


def test_changed_client_storage_keys():
    """Only the client-storage entries a round wrote are shared across ranks:
    rebound entries, tensors changed in place, and mutable objects."""
    import torch

    from fedsim_amd.distributed.centralized.centralized_fl_algorithm import (
        _changed_keys, _storage_state)
    from fedsim_amd.utils import Storage

    st = Storage()
    h = torch.zeros(4)
    st.write("h", h)
    st.write("last_round", 2)
    st.write("same", torch.ones(2))
    st.write("d", {"a": 1})
    state = _storage_state(st)
    assert _changed_keys(st, state) == ["d"]  # a dict may change in place
    h.add_(1)  # in place: its version counter moves
    st.write("last_round", 3)
    st.write("new", 5)
    assert sorted(_changed_keys(st, state)) == ["d", "h", "last_round", "new"]
    from fedsim_amd.distributed.centralized.centralized_fl_algorithm import _removed_keys

    assert _removed_keys(st, state) == []
    st.remove("same")
    assert _removed_keys(st, state) == ["same"]


def test_host_route_policy(monkeypatch):
    """How a host vector reaches its slab row (aggregators._host_route):
    pageable vectors are staged, and so are pinned ones below 32 MB; staged
    vectors below 2 MB are read in place by the pack kernel, from 2 MB every
    second one goes through a DMA instead, larger ones (64 MB) and the
    caller's own pinned vectors from 32 MB always do; the _HOST_PACK switch
    forces either path (the A/B runs)."""
    from fedsim_amd.utils import aggregators as A

    MB = 1 << 20
    monkeypatch.setattr(A, "_HOST_PACK", "auto")
    assert A._host_route(False, 4 * MB) == (False, False)
    assert A._host_route(True, 4 * MB) == (False, False)
    assert A._host_route(False, 40 * MB) == (False, False)
    assert A._host_route(True, 40 * MB) == (True, True)
    assert A._host_route(False, 100 * MB) == (False, True)
    assert A._host_route(True, 100 * MB) == (True, True)
    # from 2 MB every second staged vector takes the DMA (the link shared)
    assert A._host_route(False, 4 * MB, odd=True) == (False, True)
    assert A._host_route(True, 4 * MB, odd=True) == (False, True)
    assert A._host_route(False, MB, odd=True) == (False, False)
    monkeypatch.setattr(A, "_HOST_PACK", "dma")
    assert A._host_route(False, 4 * MB) == (False, True)
    monkeypatch.setattr(A, "_HOST_PACK", "zero_copy")
    assert A._host_route(True, 100 * MB) == (True, False)


def test_server_step_device_rule():
    """A ServerStep runs on one device: its operands live there, or are
    page-locked host memory the GPU reaches at its own address
    (ops.host_mapped, checked on the GPU box by test_gpu_host_mapped.py);
    pageable host operands of a HIP step are refused, and a narrowed step
    keeps the device."""
    from fedsim_amd import ops

    assert not ops.host_mapped(torch.zeros(4)) and not ops.host_mapped(torch.zeros(0))
    assert not ops.host_mapped("not a tensor")
    with pytest.raises(ValueError, match="the step runs on cuda:0"):
        ops.ServerStep("fedavg", torch.zeros(8), lr=1.0, device="cuda:0")
    s = ops.ServerStep("fedavg", torch.zeros(8), lr=1.0, grad_out=torch.zeros(8))
    assert s.device == torch.device("cpu") and s.narrow(2, 6).device == s.device
    with pytest.raises(ValueError, match="HIP device"):
        s.apply(torch.zeros(8))


def test_host_state_step_selection():
    """fused_server_step takes the one-DMA-each-way host path exactly when
    the cloud (and the aux vector / momentum buffer it has) live in host
    memory as fp32 and the step runs on a HIP device; the device decision
    only (nothing is allocated)."""
    from fedsim_amd.distributed.centralized.training.utils import _host_state

    hip = torch.device("cuda", 0)
    cloud = torch.zeros(8)
    assert _host_state(cloud, None, None, hip)
    assert _host_state(cloud, torch.zeros(8), torch.zeros(8), hip)
    assert not _host_state(cloud, torch.zeros(8, dtype=torch.float64), None, hip)
    assert not _host_state(cloud, None, torch.zeros(8, device="meta"), hip)
    assert not _host_state(torch.zeros(8, device="meta"), None, None, hip)
    assert not _host_state(cloud, None, None, torch.device("cpu"))


def test_async_host_staging_threshold():
    """Handed-over host vectors are staged by the ingest worker from 2 MB on
    (tools/bench_host_rounds.py: config 2's 4.3 MB vectors gain, config 1's
    0.8 MB ones lose the hand-off)."""
    from fedsim_amd.utils.aggregators import _ASYNC_STAGE_MIN

    assert 199_210 < _ASYNC_STAGE_MIN <= 1_085_668


def test_hand_over_tokens_decide_borrowing():
    """serial_aggregation's ownership test is the explicit hand-over token
    plus the no-alias check; outside a hand-over round nothing is handed over
    -- not even a vector only its message references (no inference)."""
    from fedsim_amd.distributed.centralized.training import utils as U
    from fedsim_amd.utils.handover import hand_over, handover_round

    with handover_round():
        fresh = hand_over(torch.ones(8))
        assert U._handed_over(fresh)
        assert not U._handed_over(fresh)  # a token is consumed once
        assert not U._handed_over(torch.ones(8))  # no declaration: the clone
        kept = hand_over(torch.ones(8))
        view = kept[:4]  # noqa: F841 -- the client keeps a view of its output
        assert not U._handed_over(kept)
        changed = hand_over(torch.ones(8))
        changed.add_(1)  # changed after it was handed over
        assert not U._handed_over(changed)
        sliced = torch.ones(16)
        part = hand_over(sliced[:8])  # itself a view of another tensor
        assert not U._handed_over(part)
        again = hand_over(torch.ones(8))
        assert U._handed_over(again)
        alias = hand_over(again.detach())  # the same storage a second time
        assert not U._handed_over(alias)
    # outside a round hand_over is a no-op: the sole-owned vector is cloned
    msg = {"local_params": hand_over(torch.ones(8))}
    params = msg["local_params"]
    assert not U._handed_over(params)
    assert not U._handed_over(torch.ones(8))
    # the caller's own round declares it
    with handover_round():
        msg = {"local_params": hand_over(torch.ones(8))}
        assert U._handed_over(msg["local_params"])


def test_hand_over_round_scope_releases_tokens():
    import gc
    import weakref

    from fedsim_amd.utils.handover import _OPEN, hand_over, handover_round, take_token

    with handover_round():
        t = hand_over(torch.ones(4))
        ref = weakref.ref(t)
        del t
        gc.collect()
        assert ref() is None  # a token does not keep its tensor alive
        u = torch.ones(4)
        assert take_token(u) is False
    assert not _OPEN and take_token(u) is None



@pytest.mark.parametrize("how", ["auto", "torch", "memmove1", "memmove3", "memmove4", "memmove6",
                                 "memmove8"])
@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 3 * 1024 + 5, 1 << 14, (1 << 14) + 3,
                               6 * 1024 + 1, 12 * 1024 + 1, 6 * 2048 + 2])
def test_staging_copy_is_exact(monkeypatch, how, n):
    """The ingest worker's staging copy (aggregators._staging_copy) writes
    exactly the source floats for every method, size and thread split
    (page-rounded chunks, a short last chunk, sizes below one page) and
    nothing past the destination slice; strided or non-fp32 sources take
    torch's copy."""
    from fedsim_amd.utils import aggregators as A

    monkeypatch.setattr(A, "_STAGE_COPY", how)
    monkeypatch.setattr(A, "_STAGE_SPLIT_MIN", 4096)  # "auto" splits from 1024 floats
    monkeypatch.setattr(A, "_stage_pool", None)
    g = torch.Generator().manual_seed(n)
    src = torch.randn(n, generator=g)
    buf = torch.full((n + 16,), 7.25)
    A._staging_copy(buf[:n], src)
    assert torch.equal(buf[:n].view(torch.int32), src.view(torch.int32))
    assert (buf[n:] == 7.25).all()
    wide = torch.randn(2 * n + 2, generator=g)
    A._staging_copy(buf[:n + 1], wide[::2])  # strided source
    assert torch.equal(buf[:n + 1], wide[::2])
    if A._stage_pool is not None:
        A._stage_pool.shutdown()
