"""Pin the oracle: every oracle function must reproduce the reference's own
outputs (tests/golden, produced by tools/gen_golden.py importing the reference)
bit for bit.  CPU only."""
import numpy as np
import pytest

from conftest import bits, golden_cases
from oracle import ref
from oracle import vectors as V

CASES = golden_cases()
PARAM_CASES = [c for c in CASES if all(c["ok"]) and c["has_params"] and "opts" not in c]
OPT_CASES = [c for c in CASES if "opts" in c]


def _inputs(case):
    X = V.client_rows(case["dist"], case["K"], case["P"], case["seed"])
    assert V.sha256(X) == case["input_sha256"], "input generator drifted"
    return X


def _check(case, arrays, name, got):
    assert V.sha256(got) == case["outputs_sha256"][name], name
    if case["stored"]:
        np.testing.assert_array_equal(bits(got), bits(arrays[f"{case['id']}/{name}"]))


@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_oracle_reduce_matches_reference(case, golden):
    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, ok = ref.accepted(case["weights"])
    assert ok and W is not None
    assert (W == case["scalars"]["W"]) and (isinstance(W, int) == case["scalars"]["W_is_int"])
    s = ref.reduce(X[idx], ws)
    _check(case, arrays, "sum", s)
    _check(case, arrays, "avg", ref.reduce(X[idx], ws, W=W))
    _check(case, arrays, "avg", ref.finalize(s, W))
    if case["P"] <= 5000:
        np.testing.assert_array_equal(bits(ref.reduce_numpy(X[idx], ws)), bits(s))
        np.testing.assert_array_equal(bits(ref.finalize_numpy(s, W)), bits(ref.finalize(s, W)))


@pytest.mark.parametrize("case", PARAM_CASES, ids=[c["id"] for c in PARAM_CASES])
def test_oracle_optimize_matches_reference(case, golden):
    _, arrays = golden
    X = _inputs(case)
    idx, ws, W, _ = ref.accepted(case["weights"])
    avg = ref.reduce(X[idx], ws, W=W)
    cloud0 = V.cloud_vector(case["P"], case["seed"] + 1)
    for lr in case["lrs"]:
        if case["algo"] == "adabest":
            prev0 = V.cloud_vector(case["P"], case["seed"] + 2)
            c, ap = ref.adabest_sgd(avg, cloud0, prev0, case["beta"], lr)
            _check(case, arrays, f"avg_params_lr{lr}", ap)
        elif case["algo"] == "feddyn":
            h0 = V.cloud_vector(case["P"], case["seed"] + 3)
            c, h, ap = ref.feddyn_sgd(avg, cloud0, h0, W, case["num_clients"], lr)
            _check(case, arrays, f"h_lr{lr}", h)
            _check(case, arrays, f"avg_params_lr{lr}", ap)
        else:
            c = ref.fedavg_sgd(avg, cloud0, lr)
        _check(case, arrays, f"cloud_lr{lr}", c)


def opt_case_inputs(case):
    """Round inputs of an optimizer case (tools/gen_golden.py run_opt_case)."""
    X1 = V.client_rows(case["dist"], case["K"], case["P"], case["seed"])
    assert V.sha256(X1) == case["input_sha256"]
    X2 = V.client_rows(case["dist"], case["K"], case["P"], case["seed"] + 50)
    w = list(case["weights"])
    if case["algo"] in ("adabest", "feddyn"):
        w = [1] * case["K"]
    aux, coef = None, 0.0
    if case["algo"] == "adabest":
        aux, coef = V.cloud_vector(case["P"], case["seed"] + 2), case["beta"]
    elif case["algo"] == "feddyn":
        aux, coef = V.cloud_vector(case["P"], case["seed"] + 3), sum(w) / case["num_clients"]
    return X1, X2, w, aux, coef


@pytest.mark.parametrize("case", OPT_CASES, ids=[c["id"] for c in OPT_CASES])
def test_oracle_general_sgd_matches_reference(case, golden):
    """Two rounds with momentum / nesterov / dampening / weight decay /
    maximize server SGD: cloud per round, momentum buffer, grad, aux."""
    _, arrays = golden
    X1, X2, w, aux, coef = opt_case_inputs(case)
    W = sum(w)
    for i, opt in enumerate(case["opts"]):
        st = ref.ServerState(case["algo"], V.cloud_vector(case["P"], case["seed"] + 1), opt,
                             aux=aux, coef=coef)
        for r, X in ((1, X1), (2, X2)):
            st.step(ref.reduce(X, w, W=W))
            _check(case, arrays, f"cloud_o{i}_r{r}", st.cloud)
        if opt.get("momentum", 0):
            _check(case, arrays, f"mbuf_o{i}", st.buf)
        if case["algo"] in ("adabest",):
            _check(case, arrays, f"avg_params_o{i}", st.aux)
        if case["algo"] == "feddyn":
            _check(case, arrays, f"h_o{i}", st.aux)
            _check(case, arrays, f"avg_params_o{i}", st.avg_prev)
        _check(case, arrays, f"grad_o{i}", st.grad)


def test_oracle_edge_cases():
    by_id = {c["id"]: c for c in CASES}
    zero = [c for c in CASES if c.get("zero_at")]
    assert zero, "golden set lost its zero-weight cases"
    for c in zero:
        idx, ws, W, ok = ref.accepted(c["weights"])
        assert ok
        assert c["has_params"] == (W is not None)
        if W is None:
            assert c["reports"] == {}
    div = [c for c in CASES if c.get("diverged_at") is not None]
    assert div
    for c in div:
        diverged = [k == c["diverged_at"] for k in range(c["K"])]
        _, _, _, ok = ref.accepted(c["weights"], diverged)
        assert not ok and c["ok"][-1] is False and len(c["ok"]) == c["diverged_at"] + 1
    assert by_id


@pytest.mark.parametrize("case", [c for c in PARAM_CASES if c["P"] <= 70_000][:40],
                         ids=lambda c: c["id"])
def test_reference_aggregator_restatement_matches_reference(case, golden):
    """oracle.reference_loop.ReferenceSerialAggregator (the host leg of
    tools/bench_host_rounds.py) gives the reference's own sum and average."""
    import torch

    from oracle.reference_loop import ReferenceSerialAggregator

    _, arrays = golden
    X = _inputs(case)
    agg = ReferenceSerialAggregator()
    for k, w in enumerate(case["weights"]):
        if w > 0:
            agg.add("p", torch.from_numpy(X[k].copy()).clone(), w)
    _check(case, arrays, "sum", agg.get_sum("p").numpy())
    _check(case, arrays, "avg", agg.pop("p").numpy())
    assert "p" not in agg
