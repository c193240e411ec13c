"""Property tests of the oracle (CPU, no GPU): its three independent
restatements of the reference arithmetic agree bit for bit on random inputs.

  * oracle/fedagg_ref.c      plain C, -ffp-contract=off (the GPU suite's checker)
  * oracle/ref.py numpy twin numpy fp32 ops
  * oracle/reference_loop.py the reference's own ATen CPU op sequence
    (aggregators.py:17-40, 118-122; training/utils.py:34)

plus the size-independent properties the GPU suite relies on at full size:
chaining batches through the accumulator equals one pass, and doubling every
weight doubles the sum exactly (a power-of-two scale).
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import bits
from oracle import ref
from oracle.reference_loop import aggregate_round

# the "wide" inputs overflow to +-inf on purpose
pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")

SETTINGS = settings(max_examples=80, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@st.composite
def rounds(draw, max_k=24, max_p=300, kinds=("normal", "realistic", "wide", "special")):
    K = draw(st.integers(0, max_k))
    P = draw(st.integers(1, max_p))
    seed = draw(st.integers(0, 2**31 - 1))
    rng = np.random.default_rng(seed)
    kind = draw(st.sampled_from(list(kinds)))
    if kind == "normal":
        X = rng.standard_normal((K, P))
    elif kind == "realistic":
        X = rng.normal(0, 0.05, P) + rng.normal(0, 1e-3, (K, P))
    elif kind == "wide":
        X = rng.standard_normal((K, P)) * 10.0 ** rng.integers(-30, 30, (K, P))
    else:
        pool = np.array([0.0, -0.0, 1e-45, -1e-45, 1.1754942e-38, 3e30, -3e30, 1.0, -1.0])
        X = rng.choice(pool, (K, P))
    wkind = draw(st.sampled_from(["int", "float", "big"]))
    if wkind == "int":
        w = [int(v) for v in rng.integers(0, 601, K)]
    elif wkind == "float":
        w = [float(v) for v in rng.uniform(0.0, 40.0, K)]
    else:
        w = [int(v) for v in rng.integers(2**24, 2**26, K)]
    return X.astype(np.float32), w


def _accepted(X, w):
    keep = [k for k in range(len(w)) if w[k] > 0]
    return X[keep], [w[k] for k in keep]


@SETTINGS
@given(rounds())
def test_three_restatements_agree(r):
    X, w = r
    Xa, wa = _accepted(X, w)
    W = sum(wa)
    c_sum = ref.reduce(Xa, wa)
    np_sum = ref.reduce_numpy(Xa, wa)
    np.testing.assert_array_equal(bits(c_sum), bits(np_sum))
    t_sum, t_w = aggregate_round([torch.from_numpy(x.copy()) for x in X], w, ret_sum=True)
    assert t_w == W
    if len(wa):
        np.testing.assert_array_equal(bits(c_sum), bits(t_sum.numpy()))
        c_avg = ref.reduce(Xa, wa, W=W)
        np.testing.assert_array_equal(bits(c_avg), bits(ref.finalize(c_sum, W)))
        np.testing.assert_array_equal(bits(c_avg), bits(ref.finalize_numpy(np_sum, W)))
        t_avg = aggregate_round([torch.from_numpy(x.copy()) for x in X], w)
        np.testing.assert_array_equal(bits(c_avg), bits(t_avg.numpy()))
    else:
        assert not c_sum.any() and not np.signbit(c_sum).any()  # +0.0 start


@SETTINGS
@given(rounds(max_k=30), st.data())
def test_chained_batches_equal_one_pass(r, data):
    X, w = r
    Xa, wa = _accepted(X, w)
    if not len(wa):
        return
    cuts = sorted(set(data.draw(st.lists(st.integers(1, len(wa)), max_size=5)) + [len(wa)]))
    acc, k0 = None, 0
    for k1 in cuts:
        last = k1 == len(wa)
        acc = ref.reduce(Xa[k0:k1], wa[k0:k1], acc_in=acc, W=sum(wa) if last else None)
        k0 = k1
    np.testing.assert_array_equal(bits(acc), bits(ref.reduce(Xa, wa, W=sum(wa))))


@SETTINGS
@given(rounds(max_k=16, kinds=("normal", "realistic")))
def test_power_of_two_weight_scaling_is_exact(r):
    """Exact while no product or partial sum leaves the normal range (a
    subnormal product loses bits that its doubled twin keeps), which holds
    for the normal-range client updates this property is applied to at full
    size (tests/test_gpu_aggregator.py::test_full_size_properties)."""
    X, w = r
    Xa, wa = _accepted(X, w)
    if not len(wa) or max(wa) >= 2**25:
        return
    s1 = ref.reduce(Xa, wa)
    s2 = ref.reduce(Xa, [2 * v for v in wa])
    finite = np.isfinite(s1 * np.float32(2))
    np.testing.assert_array_equal(bits((s1 * np.float32(2))[finite]), bits(s2[finite]))


@pytest.mark.parametrize("algo", ["fedavg", "adabest", "feddyn"])
@SETTINGS
@given(P=st.integers(1, 200), seed=st.integers(0, 2**31 - 1),
       lr=st.floats(0.01, 2.0), m=st.sampled_from([0.0, 0.5, 0.9]),
       wd=st.sampled_from([0.0, 1e-4, 0.01]))
def test_server_step_plain_sgd_matches_dedicated_epilogues(algo, P, seed, lr, m, wd):
    """The general step (ref_server_step_f32) with momentum = wd = 0 equals the
    dedicated plain-SGD epilogues; with momentum it equals torch.optim.SGD on
    CPU run on the same pseudo-gradient."""
    rng = np.random.default_rng(seed)
    avg, cloud, aux = (rng.normal(0, 0.05, P).astype(np.float32) for _ in range(3))
    coef = {"fedavg": 0.0, "adabest": 0.6, "feddyn": 0.25}[algo]
    s = ref.ServerState(algo, cloud, dict(lr=lr, momentum=m, weight_decay=wd),
                        aux=None if algo == "fedavg" else aux, coef=coef)
    s.step(avg)
    # torch.optim.SGD on the pseudo-gradient the oracle produced
    c = torch.from_numpy(cloud.copy()).requires_grad_(True)
    opt = torch.optim.SGD([c], lr=lr, momentum=m, weight_decay=wd)
    c.grad = torch.from_numpy(s.grad.copy())
    opt.step()
    np.testing.assert_array_equal(bits(s.cloud), bits(c.detach().numpy()))
    if m == 0.0 and wd == 0.0:
        if algo == "fedavg":
            exp = ref.fedavg_sgd(avg, cloud, lr)
        elif algo == "adabest":
            exp, prev = ref.adabest_sgd(avg, cloud, aux, 0.6, lr)
            np.testing.assert_array_equal(bits(s.aux), bits(prev))
        else:
            exp, h, _ = ref.feddyn_sgd(avg, cloud, aux, 1, 4, lr)
            np.testing.assert_array_equal(bits(s.aux), bits(h))
        np.testing.assert_array_equal(bits(s.cloud), bits(exp))
