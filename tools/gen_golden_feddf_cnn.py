"""Golden FedDF rounds on the reference's own CNNs, from the REFERENCE's code.

Runs the reference CentralFLAlgorithm + FedDF (feddf.py:97-144,
centralized_fl_algorithm.py:411-443) on device="cpu" with its own model
classes -- SimpleCNN2(num_classes=100) on 3x24x24 inputs and SimpleCNN on
1x28x28 (fedsim/models/simple_models.py:80-256) -- whose ``Resize`` leaf is
stubbed by a parameterless module that returns its input (torchvision is
absent here; torchvision's resize is the identity at the native size, which is
the only size fed).  K=4 synthetic clients (oracle/synthetic_fl.py), a
128-sample distillation split in batches of 64, 2 global epochs, 2 rounds.

Recorded per run (tests/golden/feddf_cnn.json + feddf_cnn.npz):
  * the reference's teacher-ensemble targets (``target_agg.get("target")``,
    feddf.py:126) of every distillation batch of every round, epoch 0 (the
    generator checks that epoch 1 recomputes the same bits);
  * the final cloud: SHA-256 of the whole vector, its float64 norm, every 8th
    element, and the classifier's weights and bias in full;
  * train()'s score report.
Build container only:  python -B tools/gen_golden_feddf_cnn.py
"""
from __future__ import annotations

import importlib
import json
import os
import random
import sys
import types
from functools import partial

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch import nn  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from gen_golden import import_reference  # noqa: E402
from oracle import synthetic_fl as S  # noqa: E402
from oracle import vectors as V  # noqa: E402

NUM_CLIENTS = 8
SAMPLE_RATE = 0.5      # K = 4 clients per round
ROUNDS = 1             # train(rounds=1) runs 2 rounds (trange(rounds + 1))
VALID = 128            # distillation samples, test_batch_size 64 -> 2 batches
GLOBAL_EPOCHS = 2
LR = 0.05
STRIDE = 8             # every 8th element of the final cloud is stored

# (id, model class, model kwargs, image shape, classes)
RUNS = [
    ("d0", "SimpleCNN2", dict(num_classes=100), (3, 24, 24), 100),
    ("d1", "SimpleCNN", dict(), (1, 28, 28), 10),
]


def _stub_torchvision():
    """torchvision.transforms.Resize as a parameterless identity leaf."""
    if "torchvision" in sys.modules:
        return
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")

    class Resize(nn.Module):
        def __init__(self, size, *args, **kwargs):
            super().__init__()
            self.size = tuple(size)

        def forward(self, x):
            assert tuple(x.shape[-2:]) == self.size, "fed at the native size only"
            return x

    tvt.Resize = Resize
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt


def run(FedDF, feddf_mod, model_cls, model_kw, shape, classes):
    targets = []  # (round, epoch, batch) -> the reference's ensemble mean

    base_agg = feddf_mod.SerialAggregator

    class Recording(base_agg):
        def get(self, key, *a, **k):
            v = super().get(key, *a, **k)
            if key == "target":
                targets.append(v.detach().clone().numpy())
            return v

    feddf_mod.SerialAggregator = Recording
    try:
        cls = S.make_algorithm(FedDF)
        dm = S.ImageDataManager(NUM_CLIENTS, shape, classes, VALID)
        random.seed(S.RANDOM_SEED)
        torch.manual_seed(S.TORCH_SEED)
        alg = cls(
            data_manager=dm, metric_logger=None, num_clients=NUM_CLIENTS,
            sample_scheme="uniform", sample_rate=SAMPLE_RATE,
            model_def=partial(model_cls, **model_kw), epochs=1,
            criterion_def="CrossEntropyScore",
            optimizer_def=partial(torch.optim.SGD, lr=LR), device="cpu",
            global_epochs=GLOBAL_EPOCHS,
        )
        scores = alg.train(rounds=ROUNDS)
    finally:
        feddf_mod.SerialAggregator = base_agg
    nb = -(-VALID // 64)
    rounds = ROUNDS + 1
    assert len(targets) == rounds * GLOBAL_EPOCHS * nb, len(targets)
    t = np.stack(targets).reshape(rounds, GLOBAL_EPOCHS, nb, *targets[0].shape)
    for e in range(1, GLOBAL_EPOCHS):  # the reference recomputes: same bits
        assert np.array_equal(t[:, e].view(np.uint32), t[:, 0].view(np.uint32))
    st = alg.get_server_storage()
    cloud = st.read("cloud_params").detach().numpy().copy()
    model = st.read("model")
    names = [n for n, _ in model.named_parameters()]
    sizes = [p.numel() for _, p in model.named_parameters()]
    tail = sizes[-2] + sizes[-1]  # classifier.weight, classifier.bias
    assert names[-2:] == ["classifier.weight", "classifier.bias"]
    arrays = dict(targets=t[:, 0].copy(), cloud_sample=cloud[::STRIDE].copy(),
                  cloud_tail=cloud[-tail:].copy())
    meta = dict(P=int(cloud.size), cloud_sha256=V.sha256(cloud),
                cloud_norm=float(np.linalg.norm(cloud.astype(np.float64))),
                scores={k: float(v) for k, v in scores.items()})
    return arrays, meta


K1000 = 1000          # teachers of the single-batch case (the size FedDF is timed at)
K1000_BATCH = 64      # one distillation batch
K1000_SEED = 41       # oracle/vectors.teacher_vectors seed
K1000_X_SEED = 90201  # the batch's input: V.gauss(seed, 64 * C*H*W)


def k1000_input(shape):
    n = K1000_BATCH * int(np.prod(shape))
    return V.gauss(K1000_X_SEED, n).astype(np.float32).reshape(K1000_BATCH, *shape)


def run_k1000(R, feddf_mod, model_cls, model_kw, shape):
    """The reference's own teacher loop over K=1000 teachers on ONE batch:
    FedDF.optimize (feddf.py:97-144) with global_epochs=1 and a one-batch
    distillation split; its ``target_agg.get("target")`` (feddf.py:126) is
    recorded.  The teachers are init cloud + seeded deltas
    (oracle/vectors.teacher_vectors), so only the [64, classes] target and
    hashes are stored."""
    from torch.utils.data import DataLoader, TensorDataset

    torch.manual_seed(S.TORCH_SEED)
    model = model_cls(**model_kw)
    init = torch.nn.utils.parameters_to_vector(model.parameters()).detach().numpy().copy()
    x = torch.from_numpy(k1000_input(shape))
    st = R["Storage"]()
    cloud = torch.from_numpy(init.copy()).requires_grad_(True)
    st.write("cloud_params", cloud)
    st.write("model", model)
    st.write("global_train_split", "valid")
    st.write("global_dataloaders",
             {"valid": DataLoader(TensorDataset(x, torch.zeros(K1000_BATCH, dtype=torch.long)),
                                  batch_size=K1000_BATCH)})
    st.write("global_epochs", 1)
    st.write("optimizer", torch.optim.SGD([cloud], lr=LR))
    st.write("lr_scheduler", None)
    st.write("device", "cpu")
    agg, app = R["SerialAggregator"](), R["AppendixAggregator"]()
    agg.add("local_params", torch.from_numpy(init.copy()), 1)
    sha = []
    for t in V.teacher_vectors(init, K1000, K1000_SEED):
        app.append("local_params", torch.from_numpy(t))
        if len(sha) < 2 or len(sha) == K1000 - 1:
            sha.append(V.sha256(t))
        else:
            sha.append(None)
    targets = []
    base_agg = feddf_mod.SerialAggregator

    class Recording(base_agg):
        def get(self, key, *a, **k):
            v = super().get(key, *a, **k)
            if key == "target":
                targets.append(v.detach().clone().numpy())
            return v

    feddf_mod.SerialAggregator = Recording
    try:
        feddf_mod.FedDF.optimize(st, agg, app)
    finally:
        feddf_mod.SerialAggregator = base_agg
    assert len(targets) == 1, len(targets)
    return targets[0], dict(init_sha256=V.sha256(init), P=int(init.size),
                            x_sha256=V.sha256(x.numpy()),
                            teacher_sha256={str(k): s for k, s in enumerate(sha) if s})


def main_k1000():
    R = import_reference("/root/reference")
    _stub_torchvision()
    models = importlib.import_module("fedsim.models.simple_models")
    feddf_mod = importlib.import_module("fedsim.distributed.centralized.training.feddf")
    torch.set_num_threads(os.cpu_count() or 1)
    manifest, arrays = [], {}
    for rid, mname, mkw, shape, classes in RUNS:
        target, meta = run_k1000(R, feddf_mod, getattr(models, mname), mkw, shape)
        assert target.shape == (K1000_BATCH, classes)
        arrays[f"{rid}/target"] = target
        manifest.append(dict(id=rid, model=mname, model_kwargs=mkw, image_shape=list(shape),
                             num_classes=classes, **meta))
        print(rid, mname, meta["P"], float(np.linalg.norm(target.astype(np.float64))))
    gd = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gd, "feddf_k1000.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_feddf_cnn.py --k1000", K=K1000,
                       batch=K1000_BATCH, teacher_seed=K1000_SEED, x_seed=K1000_X_SEED,
                       torch_seed=S.TORCH_SEED, runs=manifest), f, indent=1)
    np.savez_compressed(os.path.join(gd, "feddf_k1000.npz"), **arrays)


def main():
    if "--k1000" in sys.argv[1:]:
        return main_k1000()
    import_reference("/root/reference")
    _stub_torchvision()
    models = importlib.import_module("fedsim.models.simple_models")
    feddf_mod = importlib.import_module("fedsim.distributed.centralized.training.feddf")
    manifest, arrays = [], {}
    for rid, mname, mkw, shape, classes in RUNS:
        arr, meta = run(feddf_mod.FedDF, feddf_mod, getattr(models, mname), mkw, shape, classes)
        for k, v in arr.items():
            arrays[f"{rid}/{k}"] = v
        manifest.append(dict(id=rid, model=mname, model_kwargs=mkw, image_shape=list(shape),
                             num_classes=classes, **meta))
        print(rid, mname, meta["P"], meta["cloud_norm"], meta["scores"])
    gd = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gd, "feddf_cnn.json"), "w") as f:
        json.dump(dict(generator="tools/gen_golden_feddf_cnn.py", host=S.host_signature(),
                       num_clients=NUM_CLIENTS, sample_rate=SAMPLE_RATE, rounds=ROUNDS,
                       valid_size=VALID, global_epochs=GLOBAL_EPOCHS, lr=LR, stride=STRIDE,
                       runs=manifest), f, indent=1)
    np.savez_compressed(os.path.join(gd, "feddf_cnn.npz"), **arrays)


if __name__ == "__main__":
    main()
