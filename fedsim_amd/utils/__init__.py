"""Host-side utilities of the accelerated server path."""
from .aggregators import AppendixAggregator, DeviceAggregator, SerialAggregator
from .convert_parameters import (
    initialize_module,
    vector_to_named_parameters_like,
    vector_to_parameters_like,
    vectorize_module,
)
from .dict_ops import apply_on_dict
from .storage import Storage

__all__ = [
    "SerialAggregator",
    "DeviceAggregator",
    "AppendixAggregator",
    "Storage",
    "apply_on_dict",
    "vectorize_module",
    "initialize_module",
    "vector_to_parameters_like",
    "vector_to_named_parameters_like",
]
