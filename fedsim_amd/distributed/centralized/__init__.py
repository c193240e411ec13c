"""Centralized FL on MI355X: the round driver (``CentralFLAlgorithm``, whose
``_train`` hands every client message to the device-backed aggregator) and the
algorithm plugins of ``training``, re-exported at this level as the
reference's fedsim.distributed.centralized package does."""
from . import training
from .centralized_fl_algorithm import CentralFLAlgorithm
from .training import ALGORITHMS, AdaBest, FedAvg, FedDF, FedDyn, FedNova, FedProx

__all__ = ["training", "CentralFLAlgorithm", *ALGORITHMS]
