"""Centralized FL algorithms on the MI355X aggregation path.

Attribute lookup mirrors ``fedsim.distributed.centralized.training``
(training/__init__.py:8-23) so that a ``--algorithm FedAvg`` style resolution
(fedsim_cli/utils.py:186-192) finds the same names here.
"""
from .adabest import AdaBest
from .fedavg import FedAvg
from .feddf import FedDF
from .feddyn import FedDyn
from .fednova import FedNova
from .fedprox import FedProx
from .utils import serial_aggregation

__all__ = ["FedAvg", "AdaBest", "FedDyn", "FedNova", "FedProx", "FedDF", "serial_aggregation"]
