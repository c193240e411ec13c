"""Host-side objects around the HIP aggregation path.

* ``SerialAggregator`` — the reference's duck type (add / get / pop /
  get_sum / get_weight / pop_all / items / keys / in) backed by libfedagg:
  tensor keys are reduced in HBM, scalar keys keep the reference's host
  arithmetic.  ``DeviceAggregator`` is its tensor-only core.
* ``AppendixAggregator`` — the keep-every-value aggregator FedDF uses.
* ``Storage`` — server / client key-value memory with access protection.
* parameter packing (``vectorize_module`` ...) — flat fp32 vectors and views.
* ``set_seed`` / ``get_from_module`` — the reference's seeding and lookup
  helpers.
* ``hand_over`` — a client's declaration that it gives its vector away (the
  round driver's aggregator may then read it in place, handover.py);
  ``handover_round`` — the scope such declarations live in (the driver opens
  one per round; user code calling receive_from_client may open its own).
"""
from .aggregators import AppendixAggregator, DeviceAggregator, SerialAggregator
from .convert_parameters import (
    initialize_module,
    vector_to_named_parameters_like,
    vector_to_parameters_like,
    vectorize_module,
    vectorize_module_grads,
)
from .dict_ops import apply_on_dict
from .handover import hand_over, handover_round
from .misc import get_from_module, set_seed
from .storage import Storage

__all__ = [
    "SerialAggregator", "DeviceAggregator", "AppendixAggregator", "Storage", "apply_on_dict",
    "vectorize_module", "vectorize_module_grads", "initialize_module",
    "vector_to_parameters_like", "vector_to_named_parameters_like", "get_from_module", "set_seed",
    "hand_over", "handover_round",
]
