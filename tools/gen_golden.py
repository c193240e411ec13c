"""Generate tests/golden/ by running the REFERENCE's own aggregation code.

Runs ONLY in the build container (the reference is not on the GPU box).  The
reference package is imported read-only from /root/reference through namespace
stubs for its parents (its top-level __init__ pulls torchvision/logall, which
are absent here); bytecode writing is disabled so nothing lands in the tree.

Drives, with deterministic inputs from oracle/vectors.py:
  serial_aggregation          fedsim/distributed/centralized/training/utils.py:7-57
  SerialAggregator.add/get/get_sum/get_weight/pop/pop_all
                              fedsim/utils/aggregators.py:11-144
  FedAvg.receive_from_client  fedsim/distributed/centralized/training/fedavg.py:181-191
  FedAvg.optimize             fedsim/distributed/centralized/training/fedavg.py:193-208
  AdaBest.receive_from_client fedsim/distributed/centralized/training/adabest.py:150-170
  AdaBest.optimize            fedsim/distributed/centralized/training/adabest.py:172-189
  FedNova.receive_from_client fedsim/distributed/centralized/training/fednova.py:49-66

Writes tests/golden/manifest.json (cases, scalar outputs, SHA-256 of every
input and output array) and tests/golden/vectors.npz (full output arrays for
the cases small enough to store).

usage:  python -B tools/gen_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from oracle import vectors as V  # noqa: E402

STORE_MAX_P = 4099  # store full arrays up to this P; hashes only above


def import_reference(ref_root):
    """Stub fedsim, fedsim.distributed, fedsim.distributed.centralized as
    namespace packages pointing into the reference tree, then import the
    hot-path modules normally."""
    for name in ("fedsim", "fedsim.distributed", "fedsim.distributed.centralized"):
        if name in sys.modules:
            continue
        mod = types.ModuleType(name)
        mod.__path__ = [os.path.join(ref_root, *name.split("."))]
        sys.modules[name] = mod
    import importlib

    agg = importlib.import_module("fedsim.utils.aggregators")
    storage = importlib.import_module("fedsim.utils.storage")
    training = importlib.import_module("fedsim.distributed.centralized.training")
    tutils = importlib.import_module("fedsim.distributed.centralized.training.utils")
    return dict(
        SerialAggregator=agg.SerialAggregator,
        AppendixAggregator=agg.AppendixAggregator,
        Storage=storage.Storage,
        FedAvg=training.FedAvg,
        AdaBest=training.AdaBest,
        FedNova=training.FedNova,
        FedDyn=training.FedDyn,
        serial_aggregation=tutils.serial_aggregation,
    )


def run_case(R, case):
    K, P = case["K"], case["P"]
    X = V.client_rows(case["dist"], K, P, case["seed"])
    weights = V.client_weights(case["wkind"], K, case["seed"])
    zero_at = case.get("zero_at")
    if zero_at is not None:
        for z in zero_at:
            weights[z] = 0 if isinstance(weights[z], int) else 0.0
    algo = case["algo"]
    msgs = V.client_messages(X, weights, case.get("diverged_at"))
    storage = R["Storage"]()
    agg = R["SerialAggregator"]()
    app = R["AppendixAggregator"]()
    ok_flags = []
    for k, msg in enumerate(msgs):
        if algo == "fednova":
            # FedNova weight = n / num_steps (fednova.py:58-59); use the
            # prepared float weight directly via train_weight
            ok = R["serial_aggregation"](storage, k, msg, "train", agg, train_weight=weights[k])
        elif algo in ("adabest", "feddyn"):
            ok = R["serial_aggregation"](storage, k, msg, "train", agg, train_weight=1)
        else:
            ok = R["FedAvg"].receive_from_client(storage, k, msg, "train", agg, app)
        ok_flags.append(bool(ok))
        if not ok:
            break
    out = dict(ok=ok_flags, arrays={}, scalars={})
    out["has_params"] = "local_params" in agg
    if not all(ok_flags) or not out["has_params"]:
        out["reports"] = {k: float(v) for k, v in agg.pop_all().items()} if all(ok_flags) else None
        return X, weights, out
    W = agg.get_weight("local_params")
    out["scalars"]["W"] = W if isinstance(W, int) else float(W)
    out["scalars"]["W_is_int"] = isinstance(W, int)
    out["arrays"]["sum"] = agg.get_sum("local_params").numpy().copy()
    out["arrays"]["avg"] = agg.get("local_params").numpy().copy()

    cloud0 = V.cloud_vector(P, case["seed"] + 1)
    for lr in case.get("lrs", [1.0]):
        st = R["Storage"]()
        cloud = torch.from_numpy(cloud0.copy()).requires_grad_(True)
        st.write("cloud_params", cloud)
        st.write("optimizer", torch.optim.SGD(params=[cloud], lr=lr))
        st.write("lr_scheduler", None)
        # each optimize consumes its aggregator: rebuild an identical one
        a2 = R["SerialAggregator"]()
        for k, msg in enumerate(V.client_messages(X, weights)):
            if algo in ("adabest", "feddyn"):
                R["serial_aggregation"](st, k, msg, "train", a2, train_weight=1)
            elif algo == "fednova":
                R["serial_aggregation"](st, k, msg, "train", a2, train_weight=weights[k])
            else:
                R["serial_aggregation"](st, k, msg, "train", a2)
        if algo == "adabest":
            avg_prev0 = V.cloud_vector(P, case["seed"] + 2)
            st.write("avg_params", torch.from_numpy(avg_prev0.copy()))
            st.write("beta", case["beta"])
            reports = R["AdaBest"].optimize(st, a2, R["AppendixAggregator"]())
            out["arrays"][f"avg_params_lr{lr}"] = st.read("avg_params").numpy().copy()
        elif algo == "feddyn":
            st.write("h", torch.from_numpy(V.cloud_vector(P, case["seed"] + 3)))
            st.write("num_clients", case["num_clients"])
            reports = R["FedDyn"].optimize(st, a2, R["AppendixAggregator"]())
            out["arrays"][f"h_lr{lr}"] = st.read("h").numpy().copy()
            out["arrays"][f"avg_params_lr{lr}"] = st.read("avg_params").numpy().copy()
        else:
            reports = R["FedAvg"].optimize(st, a2, R["AppendixAggregator"]())
        out["arrays"][f"cloud_lr{lr}"] = cloud.detach().numpy().copy()
        out["reports"] = {k: float(v) for k, v in reports.items()}
    return X, weights, out


def run_opt_case(R, case):
    """Two consecutive rounds of <Algo>.optimize with a general
    torch.optim.SGD (momentum / nesterov / dampening / weight decay / maximize)
    as the server optimizer, so the momentum buffer and AdaBest's avg_params /
    FedDyn's h carry from round 1 into round 2."""
    K, P, algo = case["K"], case["P"], case["algo"]
    X1 = V.client_rows(case["dist"], K, P, case["seed"])
    X2 = V.client_rows(case["dist"], K, P, case["seed"] + 50)
    weights = V.client_weights(case["wkind"], K, case["seed"])
    out = dict(ok=[True] * K, arrays={}, scalars={}, has_params=True, reports=None)
    cls = {"fedavg": R["FedAvg"], "adabest": R["AdaBest"], "feddyn": R["FedDyn"]}[algo]
    for i, opt in enumerate(case["opts"]):
        st = R["Storage"]()
        cloud = torch.from_numpy(V.cloud_vector(P, case["seed"] + 1)).requires_grad_(True)
        optimizer = torch.optim.SGD(params=[cloud], **opt)
        st.write("cloud_params", cloud)
        st.write("optimizer", optimizer)
        st.write("lr_scheduler", None)
        if algo == "adabest":
            st.write("avg_params", torch.from_numpy(V.cloud_vector(P, case["seed"] + 2)))
            st.write("beta", case["beta"])
        if algo == "feddyn":
            st.write("h", torch.from_numpy(V.cloud_vector(P, case["seed"] + 3)))
            st.write("num_clients", case["num_clients"])
        for r, X in ((1, X1), (2, X2)):
            agg = R["SerialAggregator"]()
            for k, msg in enumerate(V.client_messages(X, weights)):
                w = 1 if algo in ("adabest", "feddyn") else None
                R["serial_aggregation"](st, k, msg, "train", agg, train_weight=w)
            cls.optimize(st, agg, R["AppendixAggregator"]())
            out["arrays"][f"cloud_o{i}_r{r}"] = cloud.detach().numpy().copy()
        if opt.get("momentum", 0):
            out["arrays"][f"mbuf_o{i}"] = optimizer.state[cloud]["momentum_buffer"].numpy().copy()
        if algo in ("adabest", "feddyn"):
            out["arrays"][f"avg_params_o{i}"] = st.read("avg_params").numpy().copy()
        if algo == "feddyn":
            out["arrays"][f"h_o{i}"] = st.read("h").numpy().copy()
        out["arrays"][f"grad_o{i}"] = cloud.grad.numpy().copy()
    return X1, weights, out


SGD_OPTS = [
    dict(lr=0.7, momentum=0.9),
    dict(lr=0.5, momentum=0.9, nesterov=True),
    dict(lr=1.0, momentum=0.5, dampening=0.1, weight_decay=1e-3),
    dict(lr=0.3, weight_decay=0.01, maximize=True),
]


def build_cases():
    cases = []
    cid = 0

    def add(**kw):
        nonlocal cid
        kw.setdefault("seed", 1000 + cid)
        kw["id"] = f"c{cid:03d}"
        cases.append(kw)
        cid += 1

    for dist in ("normal", "realistic"):
        for K in (1, 2, 3, 7, 64, 257):
            for P in (1, 3, 4, 5, 1023, 65537):
                if K * P > 4_500_000:
                    continue
                add(K=K, P=P, dist=dist, wkind="fedavg", algo="fedavg", lrs=[1.0, 0.3])
    for K, P in ((3, 1023), (64, 4099), (257, 5)):
        add(K=K, P=P, dist="realistic", wkind="adabest", algo="adabest", beta=0.6,
            lrs=[1.0, 0.3])
        add(K=K, P=P, dist="normal", wkind="fednova", algo="fednova", lrs=[1.0])
        add(K=K, P=P, dist="realistic", wkind="adabest", algo="feddyn", num_clients=37,
            lrs=[1.0, 0.3])
        add(K=K, P=P, dist="special", wkind="fedavg", algo="fedavg", lrs=[1.0, 0.3])
        add(K=K, P=P, dist="normal", wkind="bigint", algo="fedavg", lrs=[1.0])
    # edge cases of serial_aggregation (utils.py:39-46)
    add(K=5, P=1023, dist="realistic", wkind="fedavg", algo="fedavg", zero_at=[1, 3], lrs=[1.0])
    add(K=4, P=1023, dist="realistic", wkind="fedavg", algo="fedavg", zero_at=[0, 1, 2, 3],
        lrs=[1.0])
    add(K=6, P=1023, dist="realistic", wkind="fedavg", algo="fedavg", diverged_at=4, lrs=[1.0])
    # model-sized layouts (a2): SimpleMLP P=199,210 (config 1, K=5); SimpleCNN2 P=1,085,668
    add(K=5, P=199_210, dist="realistic", wkind="fedavg", algo="fedavg", lrs=[1.0])
    add(K=10, P=1_085_668, dist="realistic", wkind="fedavg", algo="fedavg", lrs=[1.0])
    add(K=10, P=1_085_668, dist="realistic", wkind="adabest", algo="adabest", beta=0.6, lrs=[1.0])
    add(K=10, P=1_085_668, dist="realistic", wkind="adabest", algo="feddyn", num_clients=1000,
        lrs=[1.0])
    # general server optimizer (momentum SGD etc.), two rounds each
    for K, P in ((7, 1023), (64, 4099)):
        add(K=K, P=P, dist="realistic", wkind="fedavg", algo="fedavg", opts=SGD_OPTS)
        add(K=K, P=P, dist="realistic", wkind="adabest", algo="adabest", beta=0.6,
            opts=SGD_OPTS)
        add(K=K, P=P, dist="realistic", wkind="adabest", algo="feddyn", num_clients=37,
            opts=SGD_OPTS)
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    a = ap.parse_args()
    torch.set_num_threads(8)
    R = import_reference(a.ref)
    os.makedirs(a.out, exist_ok=True)
    manifest = dict(
        generator="tools/gen_golden.py",
        torch=torch.__version__,
        numpy=np.__version__,
        reference="varnio/fedsim v0.9.1 @ /root/reference (imported read-only)",
        store_max_p=STORE_MAX_P,
        cases=[],
    )
    arrays = {}
    for case in build_cases():
        X, weights, out = (run_opt_case if "opts" in case else run_case)(R, case)
        entry = dict(case)
        entry["weights"] = weights
        entry["input_sha256"] = V.sha256(X)
        entry["ok"] = out["ok"]
        entry["has_params"] = out["has_params"]
        entry["scalars"] = out["scalars"]
        entry["reports"] = out.get("reports")
        entry["outputs_sha256"] = {k: V.sha256(v) for k, v in out["arrays"].items()}
        entry["stored"] = case["P"] <= STORE_MAX_P
        if entry["stored"]:
            for k, v in out["arrays"].items():
                arrays[f"{case['id']}/{k}"] = v
        manifest["cases"].append(entry)
        print(case["id"], case["K"], case["P"], case["dist"], case["wkind"], case["algo"],
              "ok" if all(out["ok"]) else "diverged", flush=True)
    with open(os.path.join(a.out, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    np.savez_compressed(os.path.join(a.out, "vectors.npz"), **arrays)
    print("cases:", len(manifest["cases"]), "arrays:", len(arrays))


if __name__ == "__main__":
    main()
