"""Golden fixtures for the dtype-generic SerialAggregator keys, from the
REFERENCE's own code.  Build container only (the reference is not on the GPU
box).

1. generic_keys: every scenario of oracle/generic_cases.py replayed through
   the reference's SerialAggregator (fedsim/utils/aggregators.py:11-144);
   the transcripts (bit-exact tensor bytes, exact numbers, raised exception
   types) go to tests/golden/generic_keys.json.
2. dtype rounds: the reference's round loop (CentralFLAlgorithm._train,
   centralized_fl_algorithm.py:411-443) over oracle/synthetic_fl.py's
   synthetic federation with an fp64 / bf16 TinyModel on device="cpu": the
   final cloud_params (+ AdaBest's avg_params, the SGD momentum buffer) and
   train()'s score report, as raw bytes in the same file.

usage: python -B tools/gen_golden_generic.py
"""
from __future__ import annotations

import importlib
import json
import os
import random
import sys
from functools import partial

sys.dont_write_bytecode = True

import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from gen_golden import import_reference  # noqa: E402
from oracle import generic_cases as G  # noqa: E402
from oracle import synthetic_fl as S  # noqa: E402

# (algorithm, model, alg kwargs, server SGD kwargs)
DTYPE_RUNS = [
    ("FedAvg", "TinyModel64", dict(), dict(lr=1.0)),
    ("FedAvg", "TinyModel64", dict(), dict(lr=0.5, momentum=0.9)),
    ("AdaBest", "TinyModel64", dict(mu=0.01, beta=0.6), dict(lr=1.0)),
    ("FedAvg", "TinyModelBF16", dict(), dict(lr=1.0)),
]


def dtype_run(training, name, model, alg_kwargs, opt_kwargs):
    cls = S.make_algorithm(getattr(training, name))
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(
        data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.MODELS[model], epochs=1,
        criterion_def="CrossEntropyScore", optimizer_def=partial(torch.optim.SGD, **opt_kwargs),
        device="cpu", **alg_kwargs,
    )
    scores = alg.train(rounds=S.ROUNDS)
    st = alg.get_server_storage()
    cloud = st.read("cloud_params")
    out = dict(cloud=G.encode(cloud.detach()))
    if name == "AdaBest":
        out["avg_params"] = G.encode(st.read("avg_params"))
    buf = st.read("optimizer").state[cloud].get("momentum_buffer")
    if buf is not None:
        out["momentum_buffer"] = G.encode(buf)
    return out, {k: G.encode(v) for k, v in scores.items()}


def main():
    R = import_reference("/root/reference")
    transcripts = {name: G.replay(R["SerialAggregator"](), steps)
                   for name, steps in G.scenarios().items()}
    training = importlib.import_module("fedsim.distributed.centralized.training")
    runs = []
    for i, (name, model, akw, okw) in enumerate(DTYPE_RUNS):
        out, scores = dtype_run(training, name, model, akw, okw)
        runs.append(dict(id=f"d{i}", algorithm=name, model=model, alg_kwargs=akw,
                         opt_kwargs=okw, outputs=out, scores=scores))
        print(f"d{i}", name, model, okw, len(scores), "scores")
    with open(os.path.join(REPO, "tests", "golden", "generic_keys.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_generic.py", transcripts=transcripts,
                       dtype_runs=runs), f, indent=0)
    print(len(transcripts), "transcripts")


if __name__ == "__main__":
    main()
