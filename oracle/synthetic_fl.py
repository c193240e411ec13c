"""Synthetic federation for round-loop parity (TEST INFRASTRUCTURE ONLY).

Used identically by tools/gen_golden_rounds.py (driving the REFERENCE's
CentralFLAlgorithm._train, centralized_fl_algorithm.py:411-443) and by
tests/test_gpu_roundloop.py (driving fedsim_amd's): a fake DataManager, a tiny
model, and a deterministic ``send_to_server`` that returns
``cloud + delta(client, round)`` so the multi-round trajectory depends on every
aggregation and server step.  No datasets, no local training.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn
from torch.nn.utils import parameters_to_vector
from torch.utils.data import TensorDataset

from fedsim_amd.utils.handover import hand_over

from . import vectors as V

NUM_CLIENTS = 20
SAMPLE_RATE = 0.25
ROUNDS = 4  # train(rounds=4) runs 5 rounds (trange(rounds + 1), :415)
RANDOM_SEED = 123
TORCH_SEED = 0


class FakeDataManager(object):
    def __init__(self, num_clients=NUM_CLIENTS):
        self.sizes = [int(v) for v in V.randint(4242, num_clients, 40, 400)]

    def get_global_dataset(self):
        return {}

    def get_oracle_dataset(self):
        # FedDyn.init reads len(oracle["train"]) / num_clients (feddyn.py:73-79)
        return {"train": list(range(sum(self.sizes)))}

    def get_local_dataset(self, client_id):
        return {"train": list(range(self.sizes[client_id]))}

    def get_local_splits_names(self):
        return ["train"]


class TensorDataManager(FakeDataManager):
    """FakeDataManager with real (x, y) data, for runs that keep the
    algorithm's own send_to_server (local SGD on the client) and for FedDF's
    server-side distillation split ("valid", feddf.py:66-78)."""

    def __init__(self, num_clients=NUM_CLIENTS, valid_size=0):
        super().__init__(num_clients)
        self.valid_size = valid_size

    @staticmethod
    def _data(seed, n):
        x = torch.from_numpy(V.gauss(seed, n * 37).astype(np.float32).reshape(n, 37))
        y = torch.from_numpy(V.randint(seed + 1, n, 0, 2))
        return TensorDataset(x, y)

    def get_global_dataset(self):
        return {"valid": self._data(90001, self.valid_size)} if self.valid_size else {}

    def get_local_dataset(self, client_id):
        return {"train": self._data(1000 + 2 * client_id, self.sizes[client_id])}


class TinyModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(37, 11)
        self.l2 = nn.Linear(11, 3)

    def forward(self, x):
        return self.l2(torch.relu(self.l1(x)))


class TinyModel64(TinyModel):
    """TinyModel in float64 (a model built under torch.set_default_dtype(
    torch.float64)): its parameter vector is an fp64 key of the aggregator."""

    def __init__(self):
        super().__init__()
        self.double()


class TinyModelBF16(TinyModel):
    """TinyModel in bfloat16."""

    def __init__(self):
        super().__init__()
        self.to(torch.bfloat16)


MODELS = {"TinyModel": TinyModel, "TinyModel64": TinyModel64, "TinyModelBF16": TinyModelBF16}


def synthetic_send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                             criterion, train_batch_size, inference_batch_size, optimizer_def,
                             lr_scheduler_def=None, device="cuda", ctx=None,
                             step_closure=None):
    model = ctx["model"]
    base = parameters_to_vector(model.parameters()).detach().cpu()
    delta = torch.from_numpy((0.01 * V.gauss(id * 7919 + rounds, base.numel())).astype(np.float32))
    local = base + delta.to(base.dtype)  # the model's dtype (a no-op for fp32 models)
    n = len(datasets[train_split_name])
    # a fresh vector the client keeps nowhere: declared handed over (the
    # round driver's aggregator may read it in place, fedsim_amd handover.py)
    return dict(
        local_params=hand_over(local.to(device)),
        num_steps=max(1, n // 32),
        diverged=False,
        num_samples={train_split_name: n},
        metrics={train_split_name: {"loss": 1.0 + 0.001 * id + 0.01 * rounds}},
    )


def make_algorithm(base_cls):
    """Subclass of an algorithm class with the synthetic client side."""
    return type("Synthetic" + base_cls.__name__, (base_cls,),
                {"send_to_server": synthetic_send_to_server})


def host_signature():
    """CPU model + torch's CPU kernel capability.  Dense CPU math (local SGD's
    GEMMs) rounds differently on another CPU (MKL/oneDNN pick per-ISA and
    per-vendor kernels), so runs with local training are bit-reproducible only
    on a host with the same signature as the one that made the goldens."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model} | {torch.backends.cpu.get_cpu_capability()}"


class ImageDataManager(FakeDataManager):
    """FakeDataManager whose server split holds image batches, for FedDF
    rounds on the reference's CNNs (SimpleCNN: 1 x 28 x 28, 10 classes;
    SimpleCNN2: 3 x 24 x 24, 100 classes).  Client splits are index lists:
    only their length (num_samples) is read by the synthetic client."""

    def __init__(self, num_clients, image_shape, num_classes, valid_size):
        super().__init__(num_clients)
        self.image_shape = tuple(image_shape)
        self.num_classes = num_classes
        self.valid_size = valid_size

    def get_global_dataset(self):
        n, shape = self.valid_size, self.image_shape
        x = V.gauss(90101, n * int(np.prod(shape))).astype(np.float32).reshape(n, *shape)
        y = V.randint(90102, n, 0, self.num_classes - 1)
        return {"valid": TensorDataset(torch.from_numpy(x), torch.from_numpy(y))}
