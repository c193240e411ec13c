"""FedProx on the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/fedprox.py:16-127.  The
reference class inherits FedAvg's receive_from_client / optimize / deploy /
report, so ``--algorithm FedProx`` rounds run through the same fused
reduce + server-step kernel as FedAvg.  Only the client differs (the
proximal term on every local gradient, local_updates.proximal_update); the
server additionally stores ``mu`` and ships it to each client.
"""
from __future__ import annotations

from . import local_updates
from .fedavg import FedAvg
from .utils import cloud_model_message

DEFAULT_MU = 0.0001


class FedProx(FedAvg):
    def init(server_storage, *args, **kwrag):
        FedAvg.init(server_storage)
        server_storage.write("mu", kwrag.get("mu", DEFAULT_MU))

    def send_to_client(server_storage, client_id):
        return dict(cloud_model_message(server_storage), mu=server_storage.read("mu"))

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        return local_updates.proximal_update(rounds, datasets, train_split_name, scores, epochs,
                                             criterion, train_batch_size, inference_batch_size,
                                             optimizer_def, lr_scheduler_def, device, ctx)
