"""Golden rounds of BASELINE configs 1-3 at the CLI's default participation,
from the REFERENCE's own round loop.

  cfg1  FedAvg, SimpleMLP (P = 199 210), -n 500 -c 0.01  -> K = 5
  cfg2  FedAvg, SimpleCNN2(num_classes=100) (P = 1 085 668), -n 1000 -c 0.01 -> K = 10
  cfg3  AdaBest mu:0.01 beta:0.6, same model and clients

Each runs the reference's CentralFLAlgorithm._train (centralized_fl_algorithm
.py:411-443) on device="cpu" for 3 rounds (train(rounds=2)) with the server
SGD at the CLI's default lr 1.0 (fedsim_cli/fed_learn.py:129), the reference's
own model classes (simple_models.py; torchvision's Resize stubbed as the
identity at the native size) and the synthetic clients of
oracle/synthetic_fl.py (cloud + a seeded delta: only aggregation and server
arithmetic, so the result must be bitwise).  Records SHA-256 of the final
cloud (and AdaBest's avg_params) and the score report:
tests/golden/configs.json.  Build container only:
python -B tools/gen_golden_configs.py
"""
from __future__ import annotations

import importlib
import json
import os
import random
import sys
from functools import partial

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from gen_golden import import_reference  # noqa: E402
from gen_golden_feddf_cnn import _stub_torchvision  # noqa: E402
from oracle import synthetic_fl as S  # noqa: E402
from oracle import vectors as V  # noqa: E402

ROUNDS = 2
# (id, algorithm, alg kwargs, model, model kwargs, num_clients, sample_rate)
RUNS = [
    ("cfg1", "FedAvg", {}, "SimpleMLP", {}, 500, 0.01),
    ("cfg2", "FedAvg", {}, "SimpleCNN2", dict(num_classes=100), 1000, 0.01),
    ("cfg3", "AdaBest", dict(mu=0.01, beta=0.6), "SimpleCNN2", dict(num_classes=100), 1000, 0.01),
]


def main():
    import_reference("/root/reference")
    _stub_torchvision()
    models = importlib.import_module("fedsim.models.simple_models")
    tr = importlib.import_module("fedsim.distributed.centralized.training")
    out = []
    for rid, algo, akw, mname, mkw, n, rate in RUNS:
        cls = S.make_algorithm(getattr(tr, algo))
        random.seed(S.RANDOM_SEED)
        torch.manual_seed(S.TORCH_SEED)
        alg = cls(data_manager=S.FakeDataManager(n), metric_logger=None, num_clients=n,
                  sample_scheme="uniform", sample_rate=rate,
                  model_def=partial(getattr(models, mname), **mkw), epochs=1,
                  criterion_def="CrossEntropyScore",
                  optimizer_def=partial(torch.optim.SGD, lr=1.0), device="cpu", **akw)
        scores = alg.train(rounds=ROUNDS)
        st = alg.get_server_storage()
        cloud = st.read("cloud_params").detach().numpy()
        rec = dict(id=rid, algorithm=algo, alg_kwargs=akw, model=mname, model_kwargs=mkw,
                   num_clients=n, sample_rate=rate, K=int(n * rate), P=int(cloud.size),
                   cloud_sha256=V.sha256(cloud),
                   cloud_norm=float(np.linalg.norm(cloud.astype(np.float64))),
                   scores={k: float(v) for k, v in scores.items()})
        if algo == "AdaBest":
            rec["avg_params_sha256"] = V.sha256(st.read("avg_params").detach().numpy())
        out.append(rec)
        print(rid, algo, rec["K"], rec["P"], rec["cloud_sha256"][:16], rec["scores"])
    with open(os.path.join(REPO, "tests", "golden", "configs.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_configs.py", rounds=ROUNDS, runs=out), f,
                  indent=1)


if __name__ == "__main__":
    main()
