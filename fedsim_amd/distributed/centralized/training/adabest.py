"""AdaBest with the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/adabest.py:46-195.
  receive_from_client: serial_aggregation with train_weight=1 (unweighted mean,
      W = accepted clients), plus the running ``avg_m`` statistic (:150-170)
  optimize: h = beta*(avg_params - avg); new = avg - h; pseudo = cloud - new;
      SGD step; avg_params <- avg (:172-189) — one fused libfedagg kernel for
      plain SGD, bit-identical to the reference's torch CPU arithmetic.
"""
from __future__ import annotations

from functools import partial

import torch

from ....local import default_step_closure
from ....utils import SerialAggregator, vector_to_parameters_like, vectorize_module
from .fedavg import FedAvg
from .utils import fused_server_step, pop_average, serial_aggregation, sgd_config


class AdaBest(FedAvg):
    def init(server_storage, *args, **kwrag):
        default_mu = 0.1
        default_beta = 0.85
        FedAvg.init(server_storage)
        cloud_params = server_storage.read("cloud_params")
        server_storage.write("avg_params", cloud_params.clone().detach())
        server_storage.write("h", torch.zeros_like(cloud_params))
        server_storage.write("average_sample", 0)
        server_storage.write("mu", kwrag.get("mu", default_mu))
        server_storage.write("beta", kwrag.get("beta", default_beta))
        running_stats = SerialAggregator()  # scalar keys only: host arithmetic
        running_stats.add("avg_m", 0, 0)
        server_storage.write("running_stats", running_stats)

    def send_to_client(server_storage, client_id):
        msg = FedAvg.send_to_client(server_storage, client_id)
        msg["average_sample"] = server_storage.read("running_stats").get("avg_m")
        msg["mu"] = server_storage.read("mu")
        return msg

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        # client side (outside the accelerated path): local drift correction h
        model = ctx["model"]
        mu = ctx["mu"]
        average_sample = ctx["average_sample"]
        params_init = vectorize_module(model, clone=True, detach=True)
        h = storage.read("h")
        mu_adaptive = mu / len(datasets[train_split_name]) * average_sample * epochs

        def transform_grads_fn(model):
            if h is not None:
                for p, g_a in zip(model.parameters(),
                                  vector_to_parameters_like(mu_adaptive * -h, model.parameters())):
                    p.grad += g_a

        closure = partial(default_step_closure, transform_grads=transform_grads_fn)
        opt_res = FedAvg.send_to_server(id, rounds, storage, datasets, train_split_name, scores,
                                        epochs, criterion, train_batch_size,
                                        inference_batch_size, optimizer_def, lr_scheduler_def,
                                        device, ctx, step_closure=closure)
        pseudo_grads = params_init - vectorize_module(model, clone=True, detach=True)
        last_round = storage.read("last_round")
        if h is None:
            new_h = pseudo_grads
        else:
            if last_round is None:
                last_round = rounds - 1
            new_h = 1 / (rounds - last_round) * h + pseudo_grads
        storage.write("h", new_h)
        storage.write("last_round", rounds)
        return opt_res

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        agg_res = serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                     serial_aggregator, train_weight=1)
        n_train = client_msg["num_samples"][train_split_name]
        running_stats = server_storage.read("running_stats")
        running_stats.add("avg_m", n_train / client_msg["num_steps"], 1)
        return agg_res

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" in serial_aggregator:
            beta = server_storage.read("beta")
            optimizer = server_storage.read("optimizer")
            lr_scheduler = server_storage.read("lr_scheduler")
            cloud_params = server_storage.read("cloud_params")
            avg_params = server_storage.read("avg_params")
            cfg = sgd_config(optimizer, cloud_params)
            if cfg is not None:
                new_avg, _ = fused_server_step("adabest", cloud_params,
                                               (serial_aggregator, "local_params"), optimizer,
                                               cfg, coef=beta, aux=avg_params)
            else:
                param_avg = pop_average(serial_aggregator).to(cloud_params.device)
                h = beta * (avg_params - param_avg)
                new_params = param_avg - h
                optimizer.zero_grad()
                cloud_params.grad = cloud_params.data - new_params
                optimizer.step()
                new_avg = param_avg.detach().clone()
            if lr_scheduler is not None:
                lr_scheduler.step()
            server_storage.write("avg_params", new_avg)
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(cloud=server_storage.read("cloud_params"),
                    avg=server_storage.read("avg_params"))
