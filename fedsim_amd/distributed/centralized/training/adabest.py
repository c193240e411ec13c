"""AdaBest on the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/adabest.py:46-195.

Server side (the accelerated part):
  receive_from_client  serial_aggregation with train_weight=1, so W is the
                       number of accepted clients, plus the host-side running
                       statistic ``avg_m`` = mean of n_train / num_steps
                       (adabest.py:150-170)
  optimize             h = beta (avg_params - avg); target = avg - h;
                       cloud.grad = cloud - target; SGD step; avg_params <- avg
                       (adabest.py:172-189).  With an SGD server optimizer the
                       pop, this epilogue and the step are one libfedagg
                       launch (EpiStep<ADABEST>), bitwise equal to the
                       reference's torch CPU ops.
Client side: local_updates.drift_update (outside the HIP path).
"""
from __future__ import annotations

from ....utils import SerialAggregator
from . import local_updates
from .fedavg import FedAvg
from .utils import (
    cloud_model_message,
    fused_server_step,
    init_drift_state,
    pop_average,
    serial_aggregation,
    sgd_config,
)

DEFAULTS = dict(mu=0.1, beta=0.85)


class AdaBest(FedAvg):
    def init(server_storage, *args, **kwrag):
        FedAvg.init(server_storage)
        init_drift_state(server_storage)
        server_storage.write("average_sample", 0)
        for name, default in DEFAULTS.items():
            server_storage.write(name, kwrag.get(name, default))
        stats = SerialAggregator()  # scalar keys only: host arithmetic
        stats.add("avg_m", 0, 0)
        server_storage.write("running_stats", stats)

    def send_to_client(server_storage, client_id):
        return dict(cloud_model_message(server_storage),
                    average_sample=server_storage.read("running_stats").get("avg_m"),
                    mu=server_storage.read("mu"))

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        return local_updates.drift_update(rounds, storage, datasets, train_split_name, scores,
                                          epochs, criterion, train_batch_size,
                                          inference_batch_size, optimizer_def,
                                          lr_scheduler_def, device, ctx)

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        accepted = serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                      serial_aggregator, train_weight=1)
        steps_per_sample = client_msg["num_samples"][train_split_name] / client_msg["num_steps"]
        server_storage.read("running_stats").add("avg_m", steps_per_sample, 1)
        return accepted

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" not in serial_aggregator:
            return serial_aggregator.pop_all()
        beta = server_storage.read("beta")
        opt = server_storage.read("optimizer")
        cloud = server_storage.read("cloud_params")
        prev_avg = server_storage.read("avg_params")
        cfg = sgd_config(opt, cloud)
        if cfg is not None:
            avg, _ = fused_server_step("adabest", cloud, (serial_aggregator, "local_params"),
                                       opt, cfg, coef=beta, aux=prev_avg)
        else:
            avg = pop_average(serial_aggregator).to(cloud.device)
            target = avg - beta * (prev_avg - avg)
            opt.zero_grad()
            cloud.grad = cloud.data - target
            opt.step()
            avg = avg.detach().clone()
        sched = server_storage.read("lr_scheduler")
        if sched is not None:
            sched.step()
        server_storage.write("avg_params", avg)
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(cloud=server_storage.read("cloud_params"),
                    avg=server_storage.read("avg_params"))
