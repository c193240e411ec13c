"""Golden multi-round trajectories from the REFERENCE's own round loop.

Runs the reference CentralFLAlgorithm (centralized_fl_algorithm.py:70-498) with
FedAvg / AdaBest / FedNova over the synthetic federation in oracle/synthetic_fl.py
for ROUNDS+1 rounds on device="cpu", and records the final cloud_params (and
AdaBest avg_params) plus train()'s score report.  Build container only.

usage: python -B tools/gen_golden_rounds.py
"""
from __future__ import annotations

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
from oracle import synthetic_fl as S  # noqa: E402
from oracle import vectors as V  # noqa: E402

RUNS = [
    ("FedAvg", dict(), dict(lr=1.0)),
    ("FedAvg", dict(), dict(lr=0.3)),
    ("AdaBest", dict(mu=0.01, beta=0.6), dict(lr=1.0)),
    ("FedNova", dict(), dict(lr=0.7)),
    ("FedDyn", dict(alpha=0.05), dict(lr=0.9)),
]


def run(R, name, alg_kwargs, opt_kwargs):
    base = R[name]
    cls = S.make_algorithm(base)
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(
        data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
        criterion_def="CrossEntropyScore",
        optimizer_def=partial(torch.optim.SGD, **opt_kwargs), device="cpu", **alg_kwargs,
    )
    scores = alg.train(rounds=S.ROUNDS)
    st = alg.get_server_storage()
    out = dict(cloud=st.read("cloud_params").detach().numpy().copy())
    if name in ("AdaBest", "FedDyn"):
        out["avg_params"] = st.read("avg_params").detach().numpy().copy()
    if name == "FedDyn":
        out["h"] = st.read("h").detach().numpy().copy()
    return out, {k: float(v) for k, v in scores.items()}


def main():
    R = import_reference("/root/reference")
    import importlib

    tr = importlib.import_module("fedsim.distributed.centralized.training")
    R = dict(FedAvg=tr.FedAvg, AdaBest=tr.AdaBest, FedNova=tr.FedNova, FedDyn=tr.FedDyn)
    manifest, arrays = [], {}
    for i, (name, akw, okw) in enumerate(RUNS):
        out, scores = run(R, name, akw, okw)
        rid = f"r{i}"
        for k, v in out.items():
            arrays[f"{rid}/{k}"] = v
        manifest.append(dict(id=rid, algorithm=name, alg_kwargs=akw, opt_kwargs=okw,
                             scores=scores, sha256={k: V.sha256(v) for k, v in out.items()}))
        print(rid, name, akw, okw, len(scores), "scores")
    gd = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gd, "rounds.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_rounds.py", runs=manifest), f, indent=1)
    np.savez_compressed(os.path.join(gd, "rounds.npz"), **arrays)


if __name__ == "__main__":
    main()
