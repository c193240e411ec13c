"""Round-loop parity: fedsim_amd's CentralFLAlgorithm._train reproduces the
REFERENCE's own multi-round trajectory (tests/golden/rounds.*,
tools/gen_golden_rounds.py) for FedAvg / AdaBest / FedNova / FedDyn / FedProx /
FedDF.

Bit for bit whenever everything outside the aggregation runs the reference's
own CPU arithmetic: device="cpu" (client models, cloud and FedDF's teachers on
the host, every aggregation on the MI355X), and device="cuda" for the
synthetic-client runs of the server-only algorithms (the cloud lives in HBM;
the only arithmetic is the aggregation and server step, i.e. our kernels).

Runs that also do dense model math — local SGD of real clients, or FedDF's
teacher / distillation forwards — are bitwise only on device="cpu" on a host
whose CPU matches the one that made the goldens (oracle/synthetic_fl.py
host_signature: MKL/oneDNN GEMMs round per ISA and vendor).  On the GPU
(rocBLAS/MIOpen) or another CPU they are held to a normwise tolerance:
||cloud - golden|| <= 1e-4 ||golden|| after 5 rounds (FedDyn's h, a running
sum of cloud - avg differences, against ||cloud||), and the score report
within 1e-4 relative."""
import json
import os
import random
from functools import partial

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DIR, bits
from oracle import synthetic_fl as S

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN_DIR, "rounds.json")) as _f:
    _G = json.load(_f)
RUNS = _G["runs"]
SAME_HOST = _G.get("host") == S.host_signature()

RTOL = 1e-4


@pytest.fixture(scope="module")
def arrays():
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _bitwise(run, device):
    dense = run.get("client") == "local" or run["algorithm"] == "FedDF"
    return not dense or (device == "cpu" and SAME_HOST)


def _make(run, device):
    from fedsim_amd.distributed.centralized import training

    base = getattr(training, run["algorithm"])
    client = run.get("client", "synthetic")
    cls = S.make_algorithm(base) if client == "synthetic" else base
    valid = run.get("valid_size", 0)
    dm = S.TensorDataManager(valid_size=valid) if (client == "local" or valid) \
        else S.FakeDataManager()
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    return cls(
        data_manager=dm, metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
        criterion_def="CrossEntropyScore",
        optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device=device,
        **run["alg_kwargs"],
    )


@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("run", RUNS, ids=[f"{r['id']}-{r['algorithm']}" for r in RUNS])
def test_round_loop_matches_reference(run, device, arrays):
    alg = _make(run, device)
    scores = alg.train(rounds=S.ROUNDS)
    st = alg.get_server_storage()
    exact = _bitwise(run, device)
    for name in ("cloud_params", "avg_params", "h"):
        key = f"{run['id']}/{'cloud' if name == 'cloud_params' else name}"
        if key not in arrays:
            continue
        t = st.read(name)
        assert t.device.type == device
        if name == "cloud_params" and device == "cpu":
            # init_cloud pins the host cloud: the step kernel updates it in
            # place over PCIe (training/utils._fused_server_step_host)
            assert t.is_pinned()
        got, want = t.detach().cpu().numpy(), arrays[key]
        if exact:
            np.testing.assert_array_equal(bits(got), bits(want))
        else:
            # h (FedDyn's dual vector) accumulates r * (cloud - avg), a
            # difference of two cloud-sized vectors: its rounding noise scales
            # with ||cloud||, not with its own (small) norm
            ref_norm = np.linalg.norm(arrays[f"{run['id']}/cloud"] if name == "h" else want)
            err = np.linalg.norm(got.astype(np.float64) - want) / ref_norm
            print(f"{run['id']} {run['algorithm']} {name}: normwise rel err {err:.3e}")
            assert err <= RTOL
    got_scores = {k: float(v) for k, v in scores.items()}
    if exact:
        assert got_scores == run["scores"]
    else:
        assert got_scores.keys() == run["scores"].keys()
        for k, v in run["scores"].items():
            assert got_scores[k] == pytest.approx(v, rel=RTOL), k


def test_feddf_teacher_average_is_the_exact_kernel_mean():
    """FedDF's batched teacher path: K teacher forwards in one batched
    forward (the traced replay with its Linear layers on the matrix cores,
    teacher_program.py; the vmap'd forward for models it cannot replay),
    averaged by fedagg_reduce_f32 — bitwise the reference's weight-1
    SerialAggregator mean (aggregators.py:23-60) of the SAME logits, and
    within fp32 rounding of the one-teacher-at-a-time forwards."""
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble
    from fedsim_amd.utils import vectorize_module
    from oracle import ref

    dev = torch.device("cuda")
    torch.manual_seed(5)
    model = S.TinyModel().to(dev)
    base = vectorize_module(model)
    teachers = [base + 0.05 * torch.randn_like(base) for _ in range(70)]  # > one vmap chunk
    ens = TeacherEnsemble(model, teachers, dev)
    assert ens.batched
    x = torch.randn(33, 37, device=dev)
    got = ens.mean_logits(x)
    per = torch.stack([ens._forward(t, x) for t in teachers])  # [K, B, C]
    assert ens.program is not None  # TinyModel replays: both Linear layers on MFMA
    batched = ens.program(x)
    want = ref.reduce(batched.reshape(70, -1).cpu().numpy(), [1] * 70, W=70)
    np.testing.assert_array_equal(bits(got.reshape(-1).cpu().numpy()), bits(want))
    torch.testing.assert_close(got, per.mean(0), rtol=1e-5, atol=1e-6)
    # the last teacher is left in the model, as initialize_module does
    ens.load_last()
    assert torch.equal(vectorize_module(model), teachers[-1])
