"""Algorithm plugins whose server side runs on the MI355X aggregation path.

The CLI of the reference resolves ``--algorithm <Name>`` by attribute lookup
on its training package (fedsim_cli/utils.py:186-192 over
fedsim/distributed/centralized/training/__init__.py), so every class is
exported here under the reference's name.  ``ALGORITHMS`` / ``get_algorithm``
offer the same resolution without the CLI.
"""
from .adabest import AdaBest
from .fedavg import FedAvg
from .feddf import FedDF
from .feddyn import FedDyn
from .fednova import FedNova
from .fedprox import FedProx
from .utils import serial_aggregation

ALGORITHMS = {cls.__name__: cls for cls in (FedAvg, AdaBest, FedDyn, FedNova, FedProx, FedDF)}


def get_algorithm(name: str):
    """The plugin class called ``name`` (as ``--algorithm name`` would find it)."""
    try:
        return ALGORITHMS[name]
    except KeyError:
        raise ValueError(f"unknown algorithm {name!r}; have {sorted(ALGORITHMS)}") from None


__all__ = [*ALGORITHMS, "serial_aggregation", "ALGORITHMS", "get_algorithm"]
