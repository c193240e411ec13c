"""FedProx on the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/fedprox.py:16-127.  The
server side IS FedAvg's (fedprox.py inherits receive_from_client / optimize /
deploy / report), so ``--algorithm FedProx`` rounds go through the same fused
reduce + server-step kernel.  Only the client differs: local SGD with the
proximal term ``mu * 0.5 * (params - params_init)`` added to every gradient
before clipping (fedprox.py:101-111).
"""
from __future__ import annotations

from functools import partial

from torch.nn.utils import parameters_to_vector

from ....local import default_step_closure
from ....utils import vector_to_parameters_like, vectorize_module
from .fedavg import FedAvg


class FedProx(FedAvg):
    def init(server_storage, *args, **kwrag):
        default_mu = 0.0001
        FedAvg.init(server_storage)
        server_storage.write("mu", kwrag.get("mu", default_mu))

    def send_to_client(server_storage, client_id):
        server_msg = FedAvg.send_to_client(server_storage, client_id)
        server_msg["mu"] = server_storage.read("mu")
        return server_msg

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        model = ctx["model"]
        mu = ctx["mu"]
        params_init = vectorize_module(model, clone=True, detach=True)

        def transform_grads_fn(model):
            params = parameters_to_vector(model.parameters())
            grad_additive = 0.5 * (params - params_init)
            for p, g_a in zip(model.parameters(),
                              vector_to_parameters_like(mu * grad_additive, model.parameters())):
                p.grad += g_a

        step_closure_ = partial(default_step_closure, transform_grads=transform_grads_fn)
        return FedAvg.send_to_server(id, rounds, storage, datasets, train_split_name, scores,
                                     epochs, criterion, train_batch_size, inference_batch_size,
                                     optimizer_def, lr_scheduler_def, device, ctx,
                                     step_closure=step_closure_)
