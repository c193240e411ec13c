"""Client side (the producer of the aggregated vectors), on CPU: one client's
``send_to_server`` — local SGD through local_train / default_step_closure and
the CrossEntropyScore criterion, FedProx's proximal gradient term, AdaBest's
and FedDyn's drift terms and their client-side h over two calls — reproduces
the reference's own output bit for bit on the goldens' CPU, within 1e-5
normwise on another (tests/golden/rounds.json "clients",
made by tools/gen_golden_rounds.py from fedprox.py:68-127 / fedavg.py:88-179 /
adabest.py:97-148 / feddyn.py:104-155)."""
import json
import os
from functools import partial

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DIR, bits
from oracle import synthetic_fl as S

with open(os.path.join(GOLDEN_DIR, "rounds.json")) as _f:
    _G = json.load(_f)
CLIENTS = _G["clients"]
# bitwise on the goldens' own CPU; another CPU's GEMM kernels round differently
SAME_HOST = _G.get("host") == S.host_signature()


@pytest.fixture(scope="module")
def arrays():
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", CLIENTS, ids=[c["id"] for c in CLIENTS])
def test_send_to_server_matches_reference(case, arrays):
    from fedsim_amd import scores
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.utils import Storage

    cls = getattr(training, case["algorithm"])
    lopt = case["local_opt"]
    torch.manual_seed(S.TORCH_SEED)
    dm = S.TensorDataManager()
    alg = cls(data_manager=dm, metric_logger=None, num_clients=S.NUM_CLIENTS,
              sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel,
              epochs=2, criterion_def="CrossEntropyScore",
              local_optimizer_def=partial(torch.optim.SGD, **lopt), device="cpu",
              **case["alg_kwargs"])
    st = alg.get_server_storage()
    cid = case["client_id"]
    multi = isinstance(case["rounds"], list)  # successive calls on one client storage
    cstore = Storage() if multi else None
    for i, rounds in enumerate(case["rounds"] if multi else [case["rounds"]]):
        ctx = cls.send_to_client(st, cid)
        torch.manual_seed(1000 + cid + 17 * i)
        msg = cls.send_to_server(cid, rounds, cstore, dm.get_local_dataset(cid), "train", {},
                                 2, scores.CrossEntropyScore(), 32, 64,
                                 partial(torch.optim.SGD, **lopt), None, "cpu", ctx=ctx)
    got, want = msg["local_params"].numpy(), arrays[f"{case['id']}/local_params"]
    if multi:  # the client-side drift / dual vector h the calls left behind
        h, h_want = cstore.read("h").numpy(), arrays[f"{case['id']}/h"]
        if SAME_HOST:
            np.testing.assert_array_equal(bits(h), bits(h_want))
        else:
            assert np.linalg.norm(h.astype(np.float64) - h_want) <= 1e-5 * np.linalg.norm(h_want)
    assert msg["num_steps"] == case["num_steps"]
    assert msg["diverged"] == case["diverged"]
    assert msg["num_samples"] == case["num_samples"]
    if SAME_HOST:
        np.testing.assert_array_equal(bits(got), bits(want))
        assert msg["metrics"] == case["metrics"]
    else:
        assert np.linalg.norm(got.astype(np.float64) - want) <= 1e-5 * np.linalg.norm(want)
        for k, v in case["metrics"]["train"].items():
            assert msg["metrics"]["train"][k] == pytest.approx(v, rel=1e-5)


def test_fedprox_server_side_is_fedavg():
    """fedprox.py:16 inherits FedAvg's receive_from_client / optimize, so a
    --algorithm FedProx round runs the same fused server kernel."""
    from fedsim_amd.distributed.centralized.training import FedAvg, FedProx

    for name in ("receive_from_client", "optimize", "deploy", "report"):
        assert getattr(FedProx, name) is getattr(FedAvg, name)


def test_scores_match_reference_arithmetic():
    """scores.py:180-346: sum-reduced loss / batch; micro vs macro running
    means; KL with log targets; Accuracy hits."""
    from fedsim_amd import scores

    g = torch.Generator().manual_seed(0)
    logits = torch.randn(7, 5, generator=g)
    y = torch.randint(0, 5, (7,), generator=g)
    ce = scores.CrossEntropyScore()
    v = ce(logits, y)
    ref = torch.nn.CrossEntropyLoss(reduction="sum")(logits, y) / 7
    assert bits(v.numpy()) == bits(ref.numpy())
    ce(logits[:3], y[:3])
    s3 = torch.nn.CrossEntropyLoss(reduction="sum")(logits[:3], y[:3]).item()
    s7 = torch.nn.CrossEntropyLoss(reduction="sum")(logits, y).item()
    assert ce.get_score() == (s7 + s3) / 10
    mac = scores.CrossEntropyScore(reduction="macro")
    mac(logits, y)
    mac(logits[:3], y[:3])
    assert mac.get_score() == (s7 / 7 + s3 / 3) / 2
    acc = scores.Accuracy()
    acc(logits, y)
    assert acc.get_score() == (logits.argmax(1) == y).sum().item() / 7
    kl = scores.KLDivScore(log_target=True)
    lp, lq = torch.log_softmax(logits, 1), torch.log_softmax(logits.flip(0), 1)
    assert bits(kl(lp, lq).numpy()) == bits(
        (torch.nn.KLDivLoss(log_target=True, reduction="sum")(lp, lq) / 7).numpy())
    with pytest.raises(Exception, match="size mismatch"):
        ce(logits, y[:3])
    with pytest.raises(Exception, match="invalid log_freq"):
        scores.Accuracy(log_freq=0)
    assert scores.Score().get_score() == 0
