"""FedDF on the reference's own CNNs, pinned to the REFERENCE's outputs.

tests/golden/feddf_cnn.* were made by tools/gen_golden_feddf_cnn.py, which
runs the reference's CentralFLAlgorithm + FedDF (feddf.py:97-144) with its own
SimpleCNN2(num_classes=100) and SimpleCNN (simple_models.py:80-256; the
torchvision Resize leaf stubbed as the identity at the native size) on the
CPU: K=4 synthetic clients, a 128-sample distillation split, 2 global
epochs, 2 rounds.  Here the same rounds run through fedsim_amd's FedDF with
fedsim_amd.models' restatement of those classes (same parameter layout, same
Resize leaf position) on the MI355X, where every teacher conv / pool chain /
Linear runs on the hand-written kernels (teacher_program.py):

* round 0's ensemble targets (the teachers are the same bits on both sides:
  init cloud + the synthetic deltas) within 1e-5 normwise of the reference's
  ``target_agg.get("target")``; round 1's (teachers built on round 0's
  distilled cloud) within 1e-4;
* the final cloud within 1e-4 normwise of the reference's on every 8th
  element and on the whole classifier, its norm within 1e-4, and the score
  report within 1e-4 relative (the student's forward / backward are
  MIOpen / rocBLAS work, normwise as for r7);
* the replay was kept: the round's ``teacher_replay`` storage entry shows
  conv, pool and Linear launches and no fallback.

On device="cpu" (teachers and student on the host, aggregation on the GPU)
the cloud is bitwise the reference's on a host with the generator's CPU
signature (its SHA-256), normwise elsewhere.

Also here: the replay fallback is visible (a deliberately untraceable
forward counts one fallback, with its reason), and targets are reused across
epochs only while the batch input is the same value (a dataset with random
transforms recomputes them, as the reference does).
"""
import json
import os
import random
import warnings
from functools import partial

import numpy as np
import pytest
import torch
from torch import nn

from conftest import GOLDEN_DIR
from oracle import synthetic_fl as S
from oracle import vectors as V

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN_DIR, "feddf_cnn.json")) as _f:
    _G = json.load(_f)
SAME_HOST = _G.get("host") == S.host_signature()


@pytest.fixture(scope="module")
def golden():
    with np.load(os.path.join(GOLDEN_DIR, "feddf_cnn.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _normwise(got, want):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    return float(np.linalg.norm(got - want) / np.linalg.norm(want))


def _run(run, device, record):
    from fedsim_amd import models
    from fedsim_amd.distributed.centralized import training
    from fedsim_amd.distributed.centralized.training import feddf

    orig = feddf.TeacherEnsemble.mean_logits

    def spy(self, x):
        out = orig(self, x)
        record.append(out.detach().cpu().numpy().copy())
        return out

    feddf.TeacherEnsemble.mean_logits = spy
    try:
        cls = S.make_algorithm(training.FedDF)
        dm = S.ImageDataManager(_G["num_clients"], run["image_shape"], run["num_classes"],
                                _G["valid_size"])
        random.seed(S.RANDOM_SEED)
        torch.manual_seed(S.TORCH_SEED)
        alg = cls(
            data_manager=dm, metric_logger=None, num_clients=_G["num_clients"],
            sample_scheme="uniform", sample_rate=_G["sample_rate"],
            model_def=partial(getattr(models, run["model"]), **run["model_kwargs"]), epochs=1,
            criterion_def="CrossEntropyScore",
            optimizer_def=partial(torch.optim.SGD, lr=_G["lr"]), device=device,
            global_epochs=_G["global_epochs"],
        )
        scores = alg.train(rounds=_G["rounds"])
    finally:
        feddf.TeacherEnsemble.mean_logits = orig
    return alg, scores


@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("rid", [r["id"] for r in _G["runs"]])
def test_feddf_cnn_round_matches_reference(rid, device, golden):
    from fedsim_amd import models

    run = [r for r in _G["runs"] if r["id"] == rid][0]
    got_t = []
    alg, scores = _run(run, device, got_t)
    st = alg.get_server_storage()
    model = st.read("model")
    assert isinstance(model.resize, models.Resize)  # the reference's leaf is there

    # the ensemble targets, round by round (epoch 0; epoch 1 reuses or
    # recomputes the same values)
    want_t = golden[f"{rid}/targets"]  # [rounds, batches, B, classes]
    rounds, nb = want_t.shape[:2]
    per_round = len(got_t) // rounds
    assert per_round in (nb, nb * _G["global_epochs"]), len(got_t)
    for r in range(rounds):
        for b in range(nb):
            err = _normwise(got_t[r * per_round + b], want_t[r, b])
            print(f"{rid} {run['model']} {device} round {r} batch {b}: targets {err:.2e}")
            assert err <= (1e-5 if r == 0 else 1e-4), (r, b, err)

    cloud = st.read("cloud_params").detach().cpu().numpy()
    assert cloud.size == run["P"]
    if device == "cpu" and SAME_HOST:
        assert V.sha256(cloud) == run["cloud_sha256"]
        assert {k: float(v) for k, v in scores.items()} == run["scores"]
    stride = _G["stride"]
    e_sample = _normwise(cloud[::stride], golden[f"{rid}/cloud_sample"])
    tail = golden[f"{rid}/cloud_tail"]
    e_tail = _normwise(cloud[-tail.size:], tail)
    norm = float(np.linalg.norm(cloud.astype(np.float64)))
    print(f"{rid} {device}: cloud sample {e_sample:.2e}, classifier {e_tail:.2e}, "
          f"norm {norm:.9g} vs {run['cloud_norm']:.9g}")
    assert e_sample <= 1e-4 and e_tail <= 1e-4
    assert abs(norm - run["cloud_norm"]) <= 1e-4 * run["cloud_norm"]
    got_scores = {k: float(v) for k, v in scores.items()}
    assert got_scores.keys() == run["scores"].keys()
    for k, v in run["scores"].items():
        assert got_scores[k] == pytest.approx(v, rel=1e-4), k

    if device == "cuda":  # the teachers ran on the kernels, not the vmap fallback
        rep = st.read("teacher_replay")
        assert rep["replayed"] and rep["fallbacks"] == 0, rep
        assert rep["conv_launches"] > 0 and rep["pool_launches"] > 0, rep
        assert rep["linear_launches"] > 0, rep


class _Untraceable(nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(37, 11)
        self.l2 = nn.Linear(11, 3)

    def forward(self, x):
        h = torch.relu(self.l1(x))
        if x.shape[0] > 10 ** 9:  # shape-dependent branch in the model's own forward
            h = h * 2
        return self.l2(h)


def test_replay_fallback_is_counted_and_warned():
    """A forward torch.fx cannot trace keeps the whole-model vmap: the
    ensemble counts the fallback, says why, warns, and its mean is still the
    per-teacher average."""
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble
    from fedsim_amd.utils import vectorize_module

    dev = torch.device("cuda")
    torch.manual_seed(11)
    model = _Untraceable().to(dev)
    base = vectorize_module(model)
    teachers = [base + 0.05 * torch.randn_like(base) for _ in range(5)]
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        ens = TeacherEnsemble(model, teachers, dev)
    assert ens.program is None and ens.fallbacks == 1
    assert "does not trace" in ens.fallback_reason
    assert any("teacher replay not used" in str(w.message) for w in caught)
    x = torch.randn(9, 37, device=dev)
    got = ens.mean_logits(x)
    per = torch.stack([ens._forward(t, x) for t in teachers])
    torch.testing.assert_close(got, per.mean(0), rtol=1e-5, atol=1e-6)
    assert ens.stats()["fallbacks"] == 1 and not ens.stats()["replayed"]


@pytest.mark.parametrize("K", [4, 100])
def test_replay_first_batch_mismatch_is_counted(K):
    """A replay whose first batch disagrees with the vmap'd forward is
    dropped, counted and reported with its error; above 64 teachers the check
    compares the first and last 32 and the fallback still returns every
    teacher's vmap'd logits."""
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble
    from fedsim_amd.utils import vectorize_module

    dev = torch.device("cuda")
    torch.manual_seed(12)
    model = S.TinyModel().to(dev)
    base = vectorize_module(model)
    teachers = [base + 0.05 * torch.randn_like(base) for _ in range(K)]
    ens = TeacherEnsemble(model, teachers, dev)
    assert ens.program is not None
    rows = ens._check_rows()
    assert (rows is None) == (K <= 64) and (rows is None or rows.numel() == 64)
    real = ens.program.__call__
    ens.program.__class__ = type("Broken", (ens.program.__class__,),
                                 {"__call__": lambda self, x: real(x) * 1.01})
    x = torch.randn(8, 37, device=dev)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        got = ens.mean_logits(x)
    assert ens.program is None and ens.fallbacks == 1
    assert "first batch differs" in ens.fallback_reason
    per = torch.stack([ens._forward(t, x) for t in teachers])
    torch.testing.assert_close(got, per.mean(0), rtol=1e-5, atol=1e-6)


def test_replay_kept_on_many_teachers():
    """Above 64 teachers the sampled check keeps a correct replay, and its
    logits are every teacher's forward."""
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble
    from fedsim_amd.utils import vectorize_module

    dev = torch.device("cuda")
    torch.manual_seed(13)
    model = S.TinyModel().to(dev)
    base = vectorize_module(model)
    teachers = [base + 0.05 * torch.randn_like(base) for _ in range(130)]
    ens = TeacherEnsemble(model, teachers, dev)
    x = torch.randn(8, 37, device=dev)
    logits = ens.teacher_logits(x)
    assert ens.program is not None and ens.fallbacks == 0 and logits.shape[0] == 130
    per = torch.stack([ens._forward(t, x) for t in teachers])
    torch.testing.assert_close(logits, per, rtol=1e-5, atol=1e-6)


class _Jitter(torch.utils.data.Dataset):
    """A distillation split with a random transform: every access returns
    the sample plus fresh noise (what RandomCrop / ColorJitter do)."""

    def __init__(self, n, jitter):
        g = torch.Generator().manual_seed(3)
        self.x = torch.randn(n, 37, generator=g)
        self.jitter = jitter

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        x = self.x[i]
        if self.jitter:
            x = x + 0.1 * torch.randn(37)
        return x, 0


@pytest.mark.parametrize("jitter", [False, True])
def test_targets_reused_only_for_identical_batches(jitter):
    """global_epochs=2 over an in-order loader: with a deterministic split
    the second epoch reuses each batch's targets (one teacher pass); with a
    random transform the inputs differ and every epoch recomputes them,
    as the reference does (feddf.py:117-126)."""
    from torch.utils.data import DataLoader

    from fedsim_amd.distributed.centralized.training import feddf
    from fedsim_amd.utils import AppendixAggregator, SerialAggregator, Storage, vectorize_module

    dev = torch.device("cuda")
    torch.manual_seed(13)
    model = S.TinyModel().to(dev)
    base = vectorize_module(model)
    st = Storage()
    cloud = base.clone().requires_grad_(True)
    st.write("cloud_params", cloud)
    st.write("model", model)
    st.write("global_train_split", "valid")
    st.write("global_epochs", 2)
    st.write("optimizer", torch.optim.SGD([cloud], lr=0.01))
    st.write("lr_scheduler", None)
    st.write("device", dev)
    st.write("global_dataloaders", {"valid": DataLoader(_Jitter(96, jitter), batch_size=32)})
    agg, app = SerialAggregator(), AppendixAggregator()
    for k in range(3):
        v = base + 0.05 * torch.randn_like(base)
        app.append("local_params", v.clone())
        agg.add("local_params", v, 10 + k)
    calls = []
    orig = feddf.TeacherEnsemble.mean_logits
    feddf.TeacherEnsemble.mean_logits = lambda self, x: calls.append(1) or orig(self, x)
    try:
        feddf.FedDF.optimize(st, agg, app)
    finally:
        feddf.TeacherEnsemble.mean_logits = orig
    assert len(calls) == (6 if jitter else 3)
    assert st.read("teacher_replay")["replayed"]
