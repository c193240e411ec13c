"""FedAvg with the MI355X aggregation path.

Plugin surface identical to the reference
(fedsim/distributed/centralized/training/fedavg.py:22-256): static ``init``,
``send_to_client``, ``send_to_server``, ``receive_from_client``, ``optimize``,
``deploy``, ``report``.

On the accelerated path:
  receive_from_client -> serial_aggregation -> SerialAggregator.add
      (client vector snapshotted into HBM; reduced by libfedagg)
  optimize            -> pop (fused reduce + divide) + fused pseudo-grad / SGD
      step, any SGD configuration (fedavg.py:193-208; bit-identical to torch CPU)
"""
from __future__ import annotations

import math

from torch.utils.data import DataLoader, RandomSampler

from ....local import default_step_closure, local_inference, local_train
from ....utils import initialize_module, vectorize_module
from ..centralized_fl_algorithm import CentralFLAlgorithm
from .utils import fused_server_step, pop_average, serial_aggregation, sgd_config


class FedAvg(CentralFLAlgorithm):
    def init(server_storage):
        device = server_storage.read("device")
        model = server_storage.read("model_def")().to(device)
        params = vectorize_module(model, clone=True, detach=True)
        params.requires_grad = True
        optimizer = server_storage.read("optimizer_def")(params=[params])
        lr_scheduler = None
        lr_scheduler_def = server_storage.read("lr_scheduler_def")
        if lr_scheduler_def is not None:
            lr_scheduler = lr_scheduler_def(optimizer=optimizer)
        server_storage.write("model", model)
        server_storage.write("cloud_params", params)
        server_storage.write("optimizer", optimizer)
        server_storage.write("lr_scheduler", lr_scheduler)

    def send_to_client(server_storage, client_id):
        cloud_params = server_storage.read("cloud_params")
        model = server_storage.read("model")
        initialize_module(model, cloud_params, clone=True, detach=True)
        return dict(model=model)

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        # client side: local SGD (outside the accelerated path)
        train_set = datasets[train_split_name]
        sampler = RandomSampler(
            train_set, replacement=True,
            num_samples=math.ceil(len(train_set) / train_batch_size) * train_batch_size,
        )
        train_loader = DataLoader(train_set, batch_size=train_batch_size, sampler=sampler)
        model = ctx["model"]
        optimizer = optimizer_def(model.parameters())
        lr_scheduler = lr_scheduler_def(optimizer=optimizer) if lr_scheduler_def else None
        closure = default_step_closure if step_closure is None else step_closure
        train_scores = scores.get(train_split_name, dict())
        num_train_samples, num_steps, diverged = local_train(
            model, train_loader, epochs, 0, criterion, optimizer, lr_scheduler, device,
            closure, scores=train_scores,
        )
        metrics = {train_split_name: {n: s.get_score() for n, s in train_scores.items()}}
        if rounds % getattr(criterion, "log_freq", 1) == 0 and hasattr(criterion, "get_name"):
            metrics[train_split_name][criterion.get_name()] = criterion.get_score()
        num_samples = {train_split_name: num_train_samples}
        for split_name, split in datasets.items():
            if split_name != train_split_name and split_name in scores:
                loader = DataLoader(split, batch_size=inference_batch_size, shuffle=False)
                num_samples[split_name] = local_inference(model, loader, scores[split_name],
                                                          device=device)
                metrics[split_name] = {n: s.get_score() for n, s in scores[split_name].items()}
        return dict(local_params=vectorize_module(model), num_steps=num_steps,
                    diverged=diverged, num_samples=num_samples, metrics=metrics)

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator)

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" in serial_aggregator:
            optimizer = server_storage.read("optimizer")
            lr_scheduler = server_storage.read("lr_scheduler")
            cloud_params = server_storage.read("cloud_params")
            cfg = sgd_config(optimizer, cloud_params)
            if cfg is not None:
                # pop + pseudo-gradient + SGD step in the round's last reduce pass
                fused_server_step("fedavg", cloud_params, (serial_aggregator, "local_params"),
                                  optimizer, cfg)
            else:
                param_avg = pop_average(serial_aggregator)
                pseudo_grads = cloud_params.data - param_avg.to(cloud_params.device)
                optimizer.zero_grad()
                cloud_params.grad = pseudo_grads
                optimizer.step()
                del param_avg
            if lr_scheduler is not None:
                lr_scheduler.step()
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(avg=server_storage.read("cloud_params"))

    def report(server_storage, dataloaders, rounds, scores, metric_logger, device,
               optimize_reports, deployment_points=None):
        model = server_storage.read("model")
        scores_from_deploy, norm_reports = dict(), dict()
        norm_report_freq = 50
        if deployment_points is not None:
            for point_name, point in deployment_points.items():
                initialize_module(model, point, clone=True, detach=True)
                for split_name, loader in dataloaders.items():
                    if split_name in scores:
                        split_scores = scores[split_name]
                        local_inference(model, loader, scores=split_scores, device=device)
                        for score_name, score in split_scores.items():
                            key = f"server.{point_name}.{split_name}.{score_name}"
                            scores_from_deploy[key] = score.get_score()
                    if rounds % norm_report_freq == 0:
                        norm_reports[f"server.{point_name}.param.norm"] = point.norm().item()
        return {**scores_from_deploy, **optimize_reports, **norm_reports}

