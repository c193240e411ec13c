"""FedDyn with the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/feddyn.py:17-200.
  receive_from_client: serial_aggregation with train_weight=1 (:157-167)
  optimize: weight = get_weight; avg = pop; h = h + weight/num_clients *
      (cloud - avg); new = avg - h; SGD step toward new; avg_params <- avg;
      h stored (:169-194) — one fused libfedagg kernel for plain SGD,
      bit-identical to the reference's torch CPU arithmetic.
"""
from __future__ import annotations

from functools import partial

import torch

from ....local import default_step_closure
from ....utils import vector_to_parameters_like, vectorize_module
from .fedavg import FedAvg
from .utils import fused_server_step, pop_average, serial_aggregation, sgd_config


class FedDyn(FedAvg):
    def init(server_storage, *args, **kwrag):
        default_alpha = 0.1
        local_train_split_name = "train"
        FedAvg.init(server_storage)
        cloud_params = server_storage.read("cloud_params")
        server_storage.write("avg_params", cloud_params.clone().detach())
        server_storage.write("h", torch.zeros_like(cloud_params))
        server_storage.write("alpha", kwrag.get("alpha", default_alpha))
        print("Warning: private access violation")
        print("\tFedDyn assumes prior knowledge on the number of clients and oracle samples")
        oracle_dataset = server_storage.read("oracle_dataset")[local_train_split_name]
        num_clients = server_storage.read("num_clients")
        server_storage.write("average_sample", len(oracle_dataset) / num_clients)

    def send_to_client(server_storage, client_id):
        msg = FedAvg.send_to_client(server_storage, client_id)
        msg["average_sample"] = server_storage.read("average_sample")
        msg["alpha"] = server_storage.read("alpha")
        return msg

    def send_to_server(id, rounds, storage, datasets, train_split_name, metrics, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        # client side (outside the accelerated path): dynamic regularizer
        model = ctx["model"]
        alpha = ctx["alpha"]
        average_sample = ctx["average_sample"]
        params_init = vectorize_module(model, clone=True, detach=True)
        h = storage.read("h")
        alpha_adaptive = alpha / len(datasets[train_split_name]) * average_sample

        def transform_grads_fn(model):
            grad_additive = 0.5 * (vectorize_module(model) - params_init)
            if h is not None:
                grad_additive -= h
            for p, g_a in zip(model.parameters(), vector_to_parameters_like(
                    alpha_adaptive * grad_additive, model.parameters())):
                p.grad += g_a

        closure = partial(default_step_closure, transform_grads=transform_grads_fn)
        opt_res = FedAvg.send_to_server(id, rounds, storage, datasets, train_split_name,
                                        metrics, epochs, criterion, train_batch_size,
                                        inference_batch_size, optimizer_def, lr_scheduler_def,
                                        device, ctx, step_closure=closure)
        pseudo_grads = params_init - vectorize_module(model, clone=True, detach=True)
        storage.write("h", pseudo_grads if h is None else pseudo_grads + h)
        return opt_res

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator, train_weight=1)

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" in serial_aggregator:
            weight = serial_aggregator.get_weight("local_params")
            optimizer = server_storage.read("optimizer")
            lr_scheduler = server_storage.read("lr_scheduler")
            cloud_params = server_storage.read("cloud_params")
            h = server_storage.read("h")
            num_clients = server_storage.read("num_clients")
            server_storage.change_protection("num_clients", False, False)
            cfg = sgd_config(optimizer, cloud_params)
            if cfg is not None:
                h, new_avg = fused_server_step("feddyn", cloud_params,
                                               (serial_aggregator, "local_params"), optimizer,
                                               cfg, coef=weight / num_clients, aux=h,
                                               want_avg_prev=True)
            else:
                param_avg = pop_average(serial_aggregator).to(cloud_params.device)
                pseudo_grads = cloud_params.data - param_avg
                h = h + weight / num_clients * pseudo_grads
                new_params = param_avg - h
                optimizer.zero_grad()
                cloud_params.grad = cloud_params.data - new_params
                optimizer.step()
                new_avg = param_avg.detach().clone()
            if lr_scheduler is not None:
                lr_scheduler.step()
            server_storage.write("avg_params", new_avg)
            server_storage.write("h", h.data)
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(cloud=server_storage.read("cloud_params"),
                    avg=server_storage.read("avg_params"))
