"""Golden multi-round trajectories from the REFERENCE's own round loop.

Runs the reference CentralFLAlgorithm (centralized_fl_algorithm.py:70-498) with
FedAvg / AdaBest / FedNova / FedDyn / FedProx / FedDF over the synthetic federation in oracle/synthetic_fl.py
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

# (algorithm, alg kwargs, server SGD kwargs, client side, server split size)
#   client "synthetic": deterministic send_to_server (oracle/synthetic_fl.py)
#   client "local":     the algorithm's own send_to_server = local SGD on CPU
RUNS = [
    ("FedAvg", dict(), dict(lr=1.0), "synthetic", 0),
    ("FedAvg", dict(), dict(lr=0.3), "synthetic", 0),
    ("AdaBest", dict(mu=0.01, beta=0.6), dict(lr=1.0), "synthetic", 0),
    ("FedNova", dict(), dict(lr=0.7), "synthetic", 0),
    ("FedDyn", dict(alpha=0.05), dict(lr=0.9), "synthetic", 0),
    ("FedAvg", dict(), dict(lr=1.0), "local", 0),
    ("FedProx", dict(mu=0.05), dict(lr=1.0), "local", 0),
    ("FedDF", dict(global_epochs=2), dict(lr=0.05), "synthetic", 100),
    ("AdaBest", dict(mu=0.02, beta=0.6), dict(lr=1.0), "local", 0),
    ("FedDyn", dict(alpha=0.05), dict(lr=1.0), "local", 0),
]


def run(R, name, alg_kwargs, opt_kwargs, client, valid_size):
    base = R[name]
    cls = S.make_algorithm(base) if client == "synthetic" else base
    dm = S.TensorDataManager(valid_size=valid_size) if (client == "local" or valid_size) \
        else S.FakeDataManager()
    random.seed(S.RANDOM_SEED)
    torch.manual_seed(S.TORCH_SEED)
    alg = cls(
        data_manager=dm, metric_logger=None, num_clients=S.NUM_CLIENTS,
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


# one client's send_to_server on CPU (local SGD; FedProx adds its proximal
# gradient term, AdaBest / FedDyn their drift terms and client-side h):
# (algorithm, alg kwargs, client id, rounds, local SGD kwargs); a tuple of
# rounds calls send_to_server once per entry on the same client storage, so
# the second call sees the h the first one left (adabest.py:141-147,
# feddyn.py:150-154)
CLIENT_RUNS = [
    ("FedAvg", dict(), 3, 0, dict(lr=0.1)),
    ("FedProx", dict(mu=0.5), 3, 0, dict(lr=0.1)),
    ("FedProx", dict(mu=0.05), 11, 2, dict(lr=0.05, momentum=0.9)),
    ("AdaBest", dict(mu=0.5, beta=0.6), 5, (1, 4), dict(lr=0.1)),
    ("FedDyn", dict(alpha=0.5), 7, (0, 1), dict(lr=0.1)),
]


def client_run(R, name, alg_kwargs, cid, rounds, local_opt):
    """Server init + send_to_client + the client's send_to_server, as
    _send_to_server (centralized_fl_algorithm.py:316-345) wires them."""
    if isinstance(rounds, tuple):
        return client_run_multi(R, name, alg_kwargs, cid, rounds, local_opt)
    torch.manual_seed(S.TORCH_SEED)
    dm = S.TensorDataManager()
    alg = R[name](
        data_manager=dm, metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=2,
        criterion_def="CrossEntropyScore", local_optimizer_def=partial(torch.optim.SGD,
                                                                       **local_opt),
        device="cpu", **alg_kwargs,
    )
    st = alg.get_server_storage()
    ctx = R[name].send_to_client(st, cid)
    torch.manual_seed(1000 + cid)
    scores_mod = __import__("importlib").import_module("fedsim.scores")
    msg = R[name].send_to_server(
        cid, rounds, None, dm.get_local_dataset(cid), "train", {}, 2,
        scores_mod.CrossEntropyScore(), 32, 64, partial(torch.optim.SGD, **local_opt),
        None, "cpu", ctx=ctx)
    out = dict(local_params=msg["local_params"].detach().numpy().copy())
    meta = dict(num_steps=msg["num_steps"], diverged=msg["diverged"],
                num_samples=msg["num_samples"], metrics=msg["metrics"])
    return out, meta


def client_run_multi(R, name, alg_kwargs, cid, rounds_seq, local_opt):
    """Successive send_to_server calls of one client with a persistent client
    Storage; records the last message and the client's final h."""
    torch.manual_seed(S.TORCH_SEED)
    dm = S.TensorDataManager()
    alg = R[name](
        data_manager=dm, metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=2,
        criterion_def="CrossEntropyScore", local_optimizer_def=partial(torch.optim.SGD,
                                                                       **local_opt),
        device="cpu", **alg_kwargs,
    )
    st = alg.get_server_storage()
    storage_cls = __import__("importlib").import_module("fedsim.utils").Storage
    scores_mod = __import__("importlib").import_module("fedsim.scores")
    cstore = storage_cls()
    for i, rounds in enumerate(rounds_seq):
        ctx = R[name].send_to_client(st, cid)
        torch.manual_seed(1000 + cid + 17 * i)
        msg = R[name].send_to_server(
            cid, rounds, cstore, dm.get_local_dataset(cid), "train", {}, 2,
            scores_mod.CrossEntropyScore(), 32, 64, partial(torch.optim.SGD, **local_opt),
            None, "cpu", ctx=ctx)
    out = dict(local_params=msg["local_params"].detach().numpy().copy(),
               h=cstore.read("h").detach().numpy().copy())
    meta = dict(num_steps=msg["num_steps"], diverged=msg["diverged"],
                num_samples=msg["num_samples"], metrics=msg["metrics"])
    return out, meta


def main():
    R = import_reference("/root/reference")
    import importlib

    tr = importlib.import_module("fedsim.distributed.centralized.training")
    R = {n: getattr(tr, n) for n in ("FedAvg", "AdaBest", "FedNova", "FedDyn", "FedProx", "FedDF")}
    manifest, arrays = [], {}
    for i, (name, akw, okw, client, valid_size) in enumerate(RUNS):
        out, scores = run(R, name, akw, okw, client, valid_size)
        rid = f"r{i}"
        for k, v in out.items():
            arrays[f"{rid}/{k}"] = v
        manifest.append(dict(id=rid, algorithm=name, alg_kwargs=akw, opt_kwargs=okw,
                             client=client, valid_size=valid_size, scores=scores,
                             sha256={k: V.sha256(v) for k, v in out.items()}))
        print(rid, name, akw, okw, len(scores), "scores")
    clients = []
    for i, (name, akw, cid, rounds, lopt) in enumerate(CLIENT_RUNS):
        out, meta = client_run(R, name, akw, cid, rounds, lopt)
        rid = f"c{i}"
        for k, v in out.items():
            arrays[f"{rid}/{k}"] = v
        clients.append(dict(id=rid, algorithm=name, alg_kwargs=akw, client_id=cid,
                            rounds=list(rounds) if isinstance(rounds, tuple) else rounds,
                            local_opt=lopt, sha256=V.sha256(out["local_params"]), **meta))
        print(rid, name, akw, meta["num_steps"], meta["metrics"])
    gd = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gd, "rounds.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_rounds.py", host=S.host_signature(),
                       runs=manifest, clients=clients), f, indent=1)
    np.savez_compressed(os.path.join(gd, "rounds.npz"), **arrays)


if __name__ == "__main__":
    main()
