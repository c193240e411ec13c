"""FedAvg on the MI355X aggregation path.

The plugin surface is the reference's (fedsim/distributed/centralized/
training/fedavg.py:22-256): static ``init``, ``send_to_client``,
``send_to_server``, ``receive_from_client``, ``optimize``, ``deploy`` and
``report``, with the same signatures, storage keys and return values, so the
class resolves and runs under ``--algorithm FedAvg``.

What runs where:

* ``receive_from_client`` -> ``serial_aggregation`` -> ``SerialAggregator.add``:
  the client vector is borrowed (HBM-resident) or snapshotted into the HBM
  ring; no arithmetic happens on the host.
* ``optimize``: ``pop`` and the server optimizer's update are ONE libfedagg
  launch (the round's last reduce pass with the pseudo-gradient / SGD step in
  its epilogue) whenever the server optimizer is ``torch.optim.SGD`` over
  ``[cloud_params]``; the result is bit-identical to the reference's torch
  CPU ``pop`` + ``cloud - avg`` + ``optimizer.step()``.  Any other optimizer
  takes the reference's torch.optim route on the HIP-reduced average.
* ``send_to_server`` is the client (local SGD), outside the HIP path; see
  local_updates.py.
"""
from __future__ import annotations

from ..centralized_fl_algorithm import CentralFLAlgorithm
from . import local_updates
from .utils import (
    cloud_model_message,
    deployment_report,
    fused_server_step,
    init_cloud,
    pop_average,
    serial_aggregation,
    sgd_config,
)


def _step_cloud(server_storage, serial_aggregator):
    """pop("local_params") + pseudo-gradient + server optimizer step."""
    opt = server_storage.read("optimizer")
    cloud = server_storage.read("cloud_params")
    cfg = sgd_config(opt, cloud)
    if cfg is not None:
        fused_server_step("fedavg", cloud, (serial_aggregator, "local_params"), opt, cfg)
    else:
        avg = pop_average(serial_aggregator)
        opt.zero_grad()
        cloud.grad = cloud.data - avg.to(cloud.device)
        opt.step()
    sched = server_storage.read("lr_scheduler")
    if sched is not None:
        sched.step()


class FedAvg(CentralFLAlgorithm):
    def init(server_storage):
        init_cloud(server_storage)

    def send_to_client(server_storage, client_id):
        return cloud_model_message(server_storage)

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        return local_updates.sgd_update(rounds, datasets, train_split_name, scores, epochs,
                                        criterion, train_batch_size, inference_batch_size,
                                        optimizer_def, lr_scheduler_def, device, ctx,
                                        step_closure)

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator)

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" in serial_aggregator:
            _step_cloud(server_storage, serial_aggregator)
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(avg=server_storage.read("cloud_params"))

    def report(server_storage, dataloaders, rounds, scores, metric_logger, device,
               optimize_reports, deployment_points=None):
        return deployment_report(server_storage, dataloaders, rounds, scores, device,
                                 optimize_reports, deployment_points)
