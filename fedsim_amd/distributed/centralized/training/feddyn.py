"""FedDyn on the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/feddyn.py:17-200.

Server side (the accelerated part):
  receive_from_client  serial_aggregation with train_weight=1 (feddyn.py:157-167)
  optimize             r = get_weight / num_clients; avg = pop;
                       h <- h + r (cloud - avg); target = avg - h;
                       cloud.grad = cloud - target; SGD step; avg_params <- avg
                       (feddyn.py:169-194).  With an SGD server optimizer the
                       pop, this epilogue and the step are one libfedagg
                       launch (EpiStep<FEDDYN>), bitwise equal to the
                       reference's torch CPU ops.
Client side: local_updates.dynamic_reg_update (outside the HIP path).
"""
from __future__ import annotations

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

DEFAULT_ALPHA = 0.1
ORACLE_SPLIT = "train"


class FedDyn(FedAvg):
    def init(server_storage, *args, **kwrag):
        FedAvg.init(server_storage)
        init_drift_state(server_storage)
        server_storage.write("alpha", kwrag.get("alpha", DEFAULT_ALPHA))
        # the reference reads the oracle split size and the client count here
        # (a documented private-access violation) and says so on stdout
        print("Warning: private access violation")
        print("\tFedDyn assumes prior knowledge on the number of clients and oracle samples")
        n_oracle = len(server_storage.read("oracle_dataset")[ORACLE_SPLIT])
        server_storage.write("average_sample", n_oracle / server_storage.read("num_clients"))

    def send_to_client(server_storage, client_id):
        return dict(cloud_model_message(server_storage),
                    average_sample=server_storage.read("average_sample"),
                    alpha=server_storage.read("alpha"))

    def send_to_server(id, rounds, storage, datasets, train_split_name, metrics, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, step_closure=None):
        return local_updates.dynamic_reg_update(rounds, storage, datasets, train_split_name,
                                                metrics, epochs, criterion, train_batch_size,
                                                inference_batch_size, optimizer_def,
                                                lr_scheduler_def, device, ctx)

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator, train_weight=1)

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" not in serial_aggregator:
            return serial_aggregator.pop_all()
        ratio = serial_aggregator.get_weight("local_params") / server_storage.read("num_clients")
        server_storage.change_protection("num_clients", False, False)
        opt = server_storage.read("optimizer")
        cloud = server_storage.read("cloud_params")
        h = server_storage.read("h")
        cfg = sgd_config(opt, cloud)
        if cfg is not None:
            h, avg = fused_server_step("feddyn", cloud, (serial_aggregator, "local_params"),
                                       opt, cfg, coef=ratio, aux=h, want_avg_prev=True)
        else:
            avg = pop_average(serial_aggregator).to(cloud.device)
            h = h + ratio * (cloud.data - avg)
            opt.zero_grad()
            cloud.grad = cloud.data - (avg - h)
            opt.step()
            avg = avg.detach().clone()
        sched = server_storage.read("lr_scheduler")
        if sched is not None:
            sched.step()
        server_storage.write("avg_params", avg)
        server_storage.write("h", h.data)
        return serial_aggregator.pop_all()

    def deploy(server_storage):
        return dict(cloud=server_storage.read("cloud_params"),
                    avg=server_storage.read("avg_params"))
