"""Centralized FL algorithms on the MI355X aggregation path.

Attribute lookup mirrors ``fedsim.distributed.centralized.training`` so that a
``--algorithm FedAvg`` style resolution (fedsim_cli/utils.py:186-192) finds the
same names here.
"""
from .adabest import AdaBest
from .fedavg import FedAvg
from .feddyn import FedDyn
from .fednova import FedNova
from .utils import serial_aggregation

__all__ = ["FedAvg", "AdaBest", "FedNova", "FedDyn", "serial_aggregation"]
