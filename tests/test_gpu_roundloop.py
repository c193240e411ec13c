"""Round-loop parity: fedsim_amd's CentralFLAlgorithm._train with FedAvg /
AdaBest / FedNova over the synthetic federation reproduces the REFERENCE's own
multi-round trajectory (tests/golden/rounds.*, tools/gen_golden_rounds.py)
bit for bit — cloud on the HIP device (device-resident) and on the host."""
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
    RUNS = json.load(_f)["runs"]


@pytest.fixture(scope="module")
def arrays():
    with np.load(os.path.join(GOLDEN_DIR, "rounds.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("device", ["cuda", "cpu"])
@pytest.mark.parametrize("run", RUNS, ids=[r["id"] for r in RUNS])
def test_round_loop_matches_reference(run, device, arrays):
    from fedsim_amd.distributed.centralized import training

    cls = S.make_algorithm(getattr(training, run["algorithm"]))
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(
        data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
        criterion_def="CrossEntropyScore",
        optimizer_def=partial(torch.optim.SGD, **run["opt_kwargs"]), device=device,
        **run["alg_kwargs"],
    )
    scores = alg.train(rounds=S.ROUNDS)
    st = alg.get_server_storage()
    cloud = st.read("cloud_params")
    assert cloud.device.type == device
    np.testing.assert_array_equal(bits(cloud.detach().cpu().numpy()),
                                  bits(arrays[f"{run['id']}/cloud"]))
    for name in ("avg_params", "h"):
        key = f"{run['id']}/{name}"
        if key in arrays:
            t = st.read(name)
            assert t.device.type == device
            np.testing.assert_array_equal(bits(t.detach().cpu().numpy()), bits(arrays[key]))
    assert {k: float(v) for k, v in scores.items()} == run["scores"]
