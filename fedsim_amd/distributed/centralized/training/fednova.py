"""FedNova: FedAvg whose client weight is the float ``n_train / num_steps``
(reference: fedsim/distributed/centralized/training/fednova.py:49-66).  Same
kernel path; W is the Python float sum of those weights, rounded to fp32 once
at the divide."""
from __future__ import annotations

from .fedavg import FedAvg
from .utils import serial_aggregation


class FedNova(FedAvg):
    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        n_train = client_msg["num_samples"][train_split_name]
        weight = n_train / client_msg["num_steps"]
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator, train_weight=weight)
