"""Centralized FL: round driver + algorithms (reference:
fedsim/distributed/centralized/__init__.py)."""
from . import training
from .centralized_fl_algorithm import CentralFLAlgorithm
from .training import AdaBest, FedAvg, FedDyn, FedNova

__all__ = ["training", "CentralFLAlgorithm", "FedAvg", "AdaBest", "FedNova", "FedDyn"]
