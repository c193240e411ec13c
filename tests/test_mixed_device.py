"""Mixed-device and autograd sessions through the drop-in SerialAggregator
against the reference's arithmetic on the same inputs.

The reference's ``add`` is ``sum_v + value * weight`` (fedsim/utils/
aggregators.py:17-21, 35-40): an N-d running sum and an N-d value on
different devices raise RuntimeError there and leave the key as it was (a
0-dim CPU tensor is a scalar and broadcasts), and a value that requires grad
carries its autograd graph into the sum and the quotient (:55-60, 118-122).
The drop-in must give the same transcript: every result's bytes, dtype,
shape, device and ``requires_grad``, and every exception's type.

The checker is oracle/reference_loop.ReferenceSerialAggregator run on the
same tensors, with its ``v / w`` evaluated by ATen CPU (the reference CPU
aggregation the parity bar names; torch's HIP division by a scalar
multiplies by the reciprocal) and moved back to the sum's device, autograd
graph included.

CPU tests: ``requires_grad`` sessions on host values (the drop-in routes them
to the reference's arithmetic, no kernel), and the client-sharded
aggregator's device rule on its replicated bookkeeping.  GPU tests: HIP ->
host, host -> HIP, cuda:0 then a host tensor, 0-dim host tensors, bf16 /
fp64 HIP keys, requires_grad values in HBM, and the single-process sharded
aggregator (host values into HIP shards are one device).
"""
import base64

import numpy as np
import pytest
import torch

from oracle.reference_loop import ReferenceSerialAggregator


class CpuQuotientReference(ReferenceSerialAggregator):
    """The reference's aggregator with ``v / w`` evaluated by ATen CPU."""

    def get(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        v, w = self._members[key]
        if w is None or w == 0:
            return v
        if isinstance(v, torch.Tensor) and v.device.type == "cuda":
            return (v.cpu() / w).to(v.device)
        return v / w


def _enc(x):
    if isinstance(x, torch.Tensor):
        t = x.detach().cpu().contiguous()
        return {"t": str(t.dtype), "shape": list(t.shape), "dev": str(x.device),
                "rg": bool(x.requires_grad),
                "b64": base64.b64encode(t.reshape(-1).view(torch.uint8).numpy().tobytes()).decode()}
    if isinstance(x, dict):
        return {"d": [[k, _enc(v)] for k, v in x.items()]}
    if isinstance(x, (list, tuple)):
        return {"l": [_enc(v) for v in x]}
    if isinstance(x, float):
        return {"f": x.hex()}
    return {"r": repr(x)}


def _vec(seed, n=4099, dtype=torch.float32, rg=False, dev="cpu"):
    g = torch.Generator().manual_seed(seed)
    t = (torch.randn(n, generator=g, dtype=torch.float64) * 0.7).to(dtype).to(dev)
    return t.requires_grad_(True) if rg else t


def replay(agg, steps):
    """steps: ("add", key, value_factory, weight) | ("get"|"get_sum"|
    "get_weight"|"pop", key) | ("pop_all",) | ("in", key).  Each value is
    built fresh for each aggregator (the same seed: the same bits)."""
    out = []
    for st in steps:
        try:
            if st[0] == "add":
                agg.add(st[1], st[2](), st[3])
                res = None
            elif st[0] == "pop_all":
                res = agg.pop_all()
            elif st[0] == "in":
                res = st[1] in agg
            else:
                res = getattr(agg, st[0])(st[1])
            out.append(["ok", _enc(res)])
        except Exception as e:  # noqa: BLE001 -- the transcript records what was raised
            out.append(["raise", type(e).__name__])
    return out


def _reads(key):
    return [("get_weight", key), ("get_sum", key), ("get", key)]


def _v(seed, **kw):
    return lambda: _vec(seed, **kw)


# ---------------------------------------------------------------------------
# host sessions (no GPU): values that require grad keep the reference's
# arithmetic and its autograd graph
def _grad_scenarios(dev):
    return {
        "grad_first": [("add", "p", _v(1, rg=True, dev=dev), 3),
                       ("add", "p", _v(2, dev=dev), 5)] + _reads("p") + [("pop", "p")],
        "grad_later_f64": [("add", "p", _v(3, dtype=torch.float64, dev=dev), 3),
                           ("add", "p", _v(4, dtype=torch.float64, dev=dev), 0.25),
                           ("add", "p", _v(5, dtype=torch.float64, rg=True, dev=dev), 7)] +
        _reads("p") + [("pop", "p")],
        "grad_unweighted": [("add", "p", _v(6, rg=True, dev=dev), None),
                            ("add", "p", _v(7, rg=True, dev=dev), 2), ("pop", "p")],
        "grad_bf16": [("add", "p", _v(8, dtype=torch.bfloat16, rg=True, dev=dev), 3),
                      ("add", "p", _v(9, dtype=torch.bfloat16, dev=dev), 2.5), ("pop", "p")],
        "grad_f64_0dim_weight": [("add", "p", _v(10, dtype=torch.float64, rg=True, dev=dev),
                                  torch.tensor(301.0)),
                                 ("add", "p", _v(11, dtype=torch.float64, dev=dev), 4),
                                 ("pop_all",)],
    }


@pytest.mark.parametrize("name", sorted(_grad_scenarios("cpu")))
def test_requires_grad_host(name):
    from fedsim_amd.utils import SerialAggregator

    steps = _grad_scenarios("cpu")[name]
    want = replay(CpuQuotientReference(), steps)
    assert "'rg': True" in repr(want)  # the graph is carried
    assert replay(SerialAggregator(), steps) == want


def test_client_sharded_device_rule_cpu():
    """The client-sharded aggregator's replicated bookkeeping cannot see
    devices through its meta arithmetic: a value whose producer's device
    differs from the key's running sum raises on every rank, key unchanged;
    a 0-dim host tensor still broadcasts onto it."""
    from fedsim_amd.sharding import ClientShardedSerialAggregator, RemoteRow
    from shard_oracle import ChainOracleEntry

    agg = ClientShardedSerialAggregator(entry_factory=ChainOracleEntry)
    a, b = _vec(20), _vec(21)
    agg.add("p", a, 3)
    with pytest.raises(RuntimeError, match="same device"):
        agg.add("p", RemoteRow(a.shape, a.dtype, "cuda", 1), 5)
    assert agg.get_weight("p") == 3
    agg.add("p", b, 5)
    ref = ReferenceSerialAggregator()
    ref.add("p", a, 3)
    ref.add("p", b, 5)
    assert torch.equal(agg.get_sum("p").view(torch.int32), ref.get_sum("p").view(torch.int32))
    # a key that left the kernel (reference arithmetic) keeps the rule
    agg.add("p", torch.tensor(0.5), 1)   # a 0-dim host tensor: broadcast, no error
    ref.add("p", torch.tensor(0.5), 1)
    with pytest.raises(RuntimeError, match="same device"):
        agg.add("p", RemoteRow(a.shape, a.dtype, "cuda", 1), 5)
    assert torch.equal(agg.pop("p").view(torch.int32), ref.pop("p").view(torch.int32))


# ---------------------------------------------------------------------------
def _mixed_scenarios():
    H, D = "cpu", "cuda:0"
    sc = {
        # a HIP key meets a host vector: raises, the key keeps its rows
        "hip_then_host": [("add", "p", _v(30, dev=D), 3), ("add", "p", _v(31, dev=D), 5),
                          ("add", "p", _v(32, dev=H), 7), ("in", "p")] + _reads("p") +
        [("add", "p", _v(33, dev=D), 2)] + _reads("p") + [("pop", "p")],
        # a host key (reduced on the GPU, delivered on the host) meets a HIP vector
        "host_then_hip": [("add", "p", _v(40, dev=H), 3), ("add", "p", _v(41, dev=D), 5),
                          ("add", "p", _v(42, dev=H), 0.5)] + _reads("p") + [("pop", "p")],
        # the first add on the GPU, then host tensors of several kinds: an N-d
        # one raises, a 0-dim one broadcasts (the key leaves the kernel), and
        # an N-d host tensor still raises against the HIP running sum
        "hip_then_0dim_host": [("add", "p", _v(50, dev=D), 3),
                               ("add", "p", lambda: torch.tensor(0.25), 2),
                               ("add", "p", _v(51, dev=H), 1),
                               ("add", "p", _v(52, dev=D), 4)] + _reads("p") + [("pop", "p")],
        # weights as 0-dim host tensors on a HIP key
        "hip_0dim_weights": [("add", "p", _v(55, dev=D), torch.tensor(301.0)),
                             ("add", "p", _v(56, dev=D), torch.tensor(7, dtype=torch.int64)),
                             ("add", "p", _v(57, dev=H), torch.tensor(2.0))] + _reads("p") +
        [("pop", "p")],
        # generic dtypes in HBM (the rows_ref kernel keys)
        "bf16_hip_then_host": [("add", "b", _v(60, dtype=torch.bfloat16, dev=D), 3),
                               ("add", "b", _v(61, dtype=torch.bfloat16, dev=H), 5),
                               ("add", "b", _v(62, dtype=torch.bfloat16, dev=D), 0.5)] +
        _reads("b") + [("pop", "b")],
        "f64_host_then_hip": [("add", "d", _v(63, dtype=torch.float64, dev=H), 3),
                              ("add", "d", _v(64, dtype=torch.float64, dev=D), 5)] +
        _reads("d") + [("pop", "d")],
        # autograd in HBM
        "grad_hip_first": [("add", "g", _v(70, rg=True, dev=D), 3),
                           ("add", "g", _v(71, dev=D), 5)] + _reads("g") + [("pop", "g")],
        "grad_hip_later": [("add", "g", _v(72, dev=D), 3), ("add", "g", _v(73, dev=D), 0.1),
                           ("add", "g", _v(74, rg=True, dev=D), 7),
                           ("add", "g", _v(75, dev=D), 2)] + _reads("g") + [("pop", "g")],
        "grad_hip_bf16": [("add", "g", _v(76, dtype=torch.bfloat16, rg=True, dev=D), 3),
                          ("add", "g", _v(77, dtype=torch.bfloat16, dev=D), 5), ("pop", "g")],
        "grad_then_host": [("add", "g", _v(78, rg=True, dev=D), 3),
                           ("add", "g", _v(79, dev=H), 5)] + _reads("g") + [("pop", "g")],
        # 0-dim HIP sums (a metric kept on the GPU): ATen CPU's quotient bits
        "hip_0dim_metrics": [("add", "m", lambda: torch.tensor(0.731, device=D), 2.5),
                             ("add", "m", lambda: torch.tensor(1.9, device=D), 7),
                             ("add", "d", lambda: torch.tensor(0.1, dtype=torch.float64,
                                                               device=D), 3)] +
        _reads("m") + _reads("d") + [("pop", "m"), ("pop", "d")],
        # a whole round's mixed keys, read with pop_all
        "pop_all_mixed": [("add", "local_params", _v(80, dev=D), 37),
                          ("add", "clients.train.loss", lambda: 0.75, 37),
                          ("add", "local_params", _v(81, dev=H), 12),
                          ("add", "local_params", _v(82, dev=D), 12),
                          ("add", "clients.train.loss", lambda: torch.tensor(0.5), 12),
                          ("pop_all",)],
    }
    return sc


MIXED = _mixed_scenarios()


@pytest.mark.gpu
@pytest.mark.parametrize("max_rows", [4096, 2])
@pytest.mark.parametrize("name", sorted(MIXED))
def test_mixed_device_sessions_gpu(name, max_rows):
    """The drop-in's transcript equals the reference's on the same tensors:
    results (bytes, dtype, shape, device, requires_grad) and exception
    types, with the ring drained mid-stream (max_rows=2) or not."""
    from fedsim_amd.utils import SerialAggregator

    assert torch.cuda.is_available()
    steps = MIXED[name]
    want = replay(CpuQuotientReference(), steps)
    got = replay(SerialAggregator(max_rows=max_rows), steps)
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("borrow", [False, True])
def test_mixed_device_borrowing_aggregator_gpu(borrow):
    """The round driver's borrowing aggregator follows the same rule: a
    rejected host value is not borrowed or staged, and the HBM rows already
    held reduce as before."""
    from fedsim_amd.utils import SerialAggregator

    steps = MIXED["hip_then_host"] + MIXED["host_then_hip"]
    want = replay(CpuQuotientReference(), steps)
    assert replay(SerialAggregator(borrow=borrow, borrow_host=borrow), steps) == want


@pytest.mark.gpu
def test_sharded_devices_mode_host_values_gpu():
    """ShardedSerialAggregator(devices=[...]): host values into HIP shards
    are one device (the first value's, where results are delivered); a HIP
    value added to that key raises as the reference's host sum would, and
    the reverse.  Three shards on the one GPU of the box."""
    from fedsim_amd.sharding import ShardedSerialAggregator

    devs = ["cuda:0"] * 3
    H, D = "cpu", "cuda:0"
    steps = [("add", "p", _v(90, n=100_003, dev=H), 3), ("add", "p", _v(91, n=100_003, dev=H), 5),
             ("add", "p", _v(92, n=100_003, dev=D), 7)] + _reads("p") + [
        ("add", "p", _v(93, n=100_003, dev=H), 2), ("pop", "p"),
        ("add", "q", _v(94, n=100_003, dev=D), 3), ("add", "q", _v(95, n=100_003, dev=H), 5),
        ("add", "q", _v(96, n=100_003, dev=D), 1)] + _reads("q") + [("pop", "q")]
    want = replay(CpuQuotientReference(), steps)
    assert replay(ShardedSerialAggregator(devices=devs), steps) == want


@pytest.mark.gpu
def test_hip_quotient_tensor_weights_reduced_floats():
    """reference_quotient for bf16 / fp16 HIP sums and 0-dim host tensor
    weights: ATen CPU divides by the weight's ORIGINAL value in f32
    (div_true_kernel's original_scalar_value), not the weight rounded to the
    sum's dtype first (advisor, round 5: 301 would round to 300 in bf16;
    70000 overflows fp16)."""
    from fedsim_amd.utils.aggregators import reference_quotient

    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(11)
    for dt in (torch.bfloat16, torch.float16, torch.float32, torch.float64):
        v = (torch.randn(4099, generator=g, dtype=torch.float64) * 50).to(dt)
        for w in (torch.tensor(301.0), torch.tensor(70000.0), torch.tensor(301.0, dtype=torch.float64),
                  torch.tensor(0.1, dtype=torch.float64), torch.tensor(7), torch.tensor(3.3e38)):
            want = v / w
            q = reference_quotient(v.to(dev), w)
            assert q.dtype == want.dtype and q.device == dev, (dt, w)
            assert np.array_equal(q.cpu().view(-1).view(torch.uint8).numpy(),
                                  want.view(-1).view(torch.uint8).numpy()), (dt, w)


# ---------------------------------------------------------------------------
# random sessions: every mix of dtype, device, shape, requires_grad and
# weight kind the reference's add accepts or refuses
def _session_strategy():
    from hypothesis import strategies as st

    value = st.fixed_dictionaries({
        "dtype": st.sampled_from(["f32", "f32", "f32", "f64", "bf16"]),
        "dev": st.sampled_from(["cuda", "cuda", "cpu"]),
        "dim": st.sampled_from([1, 1, 1, 0]),
        "rg": st.sampled_from([False, False, False, True]),
        "seed": st.integers(0, 10_000),
    })
    weight = st.one_of(st.integers(1, 600), st.sampled_from([0.25, 2.5, 7.3, 0]),
                       st.sampled_from(["t301", "t2", "none"]))
    step = st.one_of(
        st.tuples(st.just("add"), st.sampled_from(["p", "q"]), value, weight),
        st.tuples(st.sampled_from(["get", "get_sum", "get_weight", "pop", "in"]),
                  st.sampled_from(["p", "q"])),
    )
    return st.lists(step, min_size=1, max_size=10)


_DT = {"f32": torch.float32, "f64": torch.float64, "bf16": torch.bfloat16}


def _materialize(steps):
    """Hypothesis steps -> replay() steps (values built fresh per replay)."""
    out = []
    for st_ in steps:
        if st_[0] != "add":
            out.append(st_)
            continue
        _, key, v, w = st_
        dt = _DT[v["dtype"]]
        n = 1031 if v["dim"] else None
        rg = v["rg"]

        def make(v=v, dt=dt, n=n, rg=rg):
            g = torch.Generator().manual_seed(v["seed"])
            t = (torch.randn(n if n else (), generator=g, dtype=torch.float64) * 0.7).to(dt)
            t = t.to("cuda:0" if v["dev"] == "cuda" else "cpu")
            return t.requires_grad_(True) if rg else t
        if w == "t301":
            w = torch.tensor(301.0)
        elif w == "t2":
            w = torch.tensor(2, dtype=torch.int64)
        elif w == "none":
            w = None
        out.append(("add", key, make, w))
    return out


@pytest.mark.gpu
def test_random_sessions_match_reference_gpu():
    """Hypothesis-generated sessions over two keys: fp32 / fp64 / bf16 values
    on the host or in HBM, N-d or 0-dim, with or without requires_grad,
    Python / 0-dim tensor / zero / None weights, reads interleaved, through
    a small ring (max_rows=2).  The drop-in's transcript must equal the
    reference restatement's on the same tensors."""
    from hypothesis import HealthCheck, given, settings

    from fedsim_amd.utils import SerialAggregator

    assert torch.cuda.is_available()

    seen = {"sessions": 0, "raise": 0, "grad": 0, "kernel_key": 0, "host_result": 0}

    @settings(max_examples=300, deadline=None, derandomize=True,
              suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
    @given(_session_strategy())
    def run(steps):
        ms = _materialize(steps)
        agg = SerialAggregator(max_rows=2)
        got = replay(agg, ms)
        assert got == replay(CpuQuotientReference(), ms)
        text = repr(got)
        seen["sessions"] += 1
        seen["raise"] += "'raise'" in text
        seen["grad"] += "'rg': True" in text
        seen["host_result"] += "'dev': 'cpu'" in text
        seen["kernel_key"] += any(type(e).__name__ == "_DeviceEntry"
                                  for e in agg._members.values())

    run()
    # the generator reached every regime it is meant to cover
    assert seen["sessions"] >= 250, seen
    assert min(seen["raise"], seen["grad"], seen["host_result"], seen["kernel_key"]) >= 10, seen
    print("random sessions:", seen)
