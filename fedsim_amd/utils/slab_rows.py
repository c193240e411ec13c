"""Client vectors produced straight into the round's HBM slab.

The reference builds each client's update with ``parameters_to_vector`` +
``clone`` (fedsim/utils/convert_parameters.py:78-94) and the server clones it
again (fedsim/distributed/centralized/training/utils.py:34) before
``SerialAggregator.add`` weighs it in.  When the client's model lives on the
GPU, this module lets the client write its parameters directly into a
reserved row of the round aggregator's column-blocked slab instead
(fedagg_pack_segments_f32: one launch, read P + write P, the traffic of the
reference's ``cat`` alone), so the round's reduction reads its rows at slab
speed and nothing else is copied:

* the round driver makes its aggregator the *round aggregator*
  (``round_aggregator``) while the clients run;
* ``reserve_round_row(key, module)`` asks it for the next row of ``key``'s
  ring and returns it as a :class:`SlabRow`; ``vectorize_module(module,
  out=row)`` packs the parameters into it;
* ``SerialAggregator.add(key, row, w)`` recognises its own reserved row and
  commits it in place (arrival order is kept: nothing else can take the row
  between the reservation and the add without first copying it out).

A :class:`SlabRow` is a real ``torch.Tensor`` of shape ``[P]`` for every other
use: any torch operation on it reads the row back into an ordinary tensor
(fedagg_unpack_row_f32, once, cached), and a row that is about to be reused,
or whose slab is released, is copied out first if the tensor is still alive.
"""
from __future__ import annotations

import contextlib
import threading
import weakref
from typing import Optional

import torch
from torch.utils._pytree import tree_map

from .. import ops

__all__ = ["SlabRow", "round_aggregator", "reserve_round_row", "current_round_aggregator"]


class SlabRow(torch.Tensor):
    """Row ``row`` of a column-blocked slab [ceil(P/C), R, C] seen as a flat
    [P] fp32 tensor (a wrapper subclass: it owns no storage of its own)."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    @staticmethod
    def __new__(cls, entry, slab: torch.Tensor, row: int, P: int):
        t = torch.Tensor._make_wrapper_subclass(cls, (P,), dtype=torch.float32,
                                                device=slab.device, requires_grad=False)
        t._entry = entry
        t._slab = slab
        t._row = row
        t._dense = None
        t._committed = False
        return t

    def materialize(self) -> torch.Tensor:
        """The row as an ordinary contiguous tensor (read back once)."""
        if self._dense is None:
            self._dense = ops.unpack_row(self._slab, self._row, self.shape[0])
            self._slab = None  # the copy no longer needs the slab
        return self._dense

    @property
    def in_slab(self) -> bool:
        """Still backed by its slab row (not yet copied out)."""
        return self._dense is None and self._slab is not None

    def __repr__(self):
        return "SlabRow(row=%d, P=%d)" % (self._row, self.shape[0])

    @classmethod
    def __torch_dispatch__(cls, func, types, args=(), kwargs=None):
        def unwrap(x):
            return x.materialize() if isinstance(x, SlabRow) else x

        return func(*tree_map(unwrap, args), **tree_map(unwrap, kwargs or {}))


_local = threading.local()


def current_round_aggregator():
    return getattr(_local, "agg", None)


@contextlib.contextmanager
def round_aggregator(agg):
    """Make ``agg`` the aggregator clients of this thread vectorize into."""
    prev = getattr(_local, "agg", None)
    _local.agg = agg
    try:
        yield agg
    finally:
        _local.agg = prev


def reserve_round_row(key: str, module) -> Optional[SlabRow]:
    """A reserved slab row of the round aggregator's ``key`` for ``module``'s
    flat parameter vector, or None when there is no round aggregator, it
    does not reserve rows, or the parameters are not fp32 tensors on one HIP
    device (the caller then vectorizes as the reference does)."""
    agg = current_round_aggregator()
    reserve = getattr(agg, "reserve", None)
    if reserve is None:
        return None
    params = list(module.parameters())
    if not params:
        return None
    dev = params[0].device
    if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in params):
        return None
    P = sum(p.numel() for p in params)
    return reserve(key, P, dev)


class RowRefs(object):
    """The SlabRows an entry handed out, by row (weak references): a row that
    is about to be written again, or a slab about to be released, copies a
    still-alive row out first."""

    def __init__(self):
        self.refs = {}

    def track(self, row: SlabRow) -> None:
        self.refs[row._row] = weakref.ref(row)

    def claim(self, r: int, slab) -> bool:
        """Row r of ``slab`` is about to be overwritten; returns True if a
        live SlabRow had to be copied out (the caller orders later copies)."""
        ref = self.refs.pop(r, None)
        row = None if ref is None else ref()
        if row is not None and row._slab is slab and row._dense is None:
            row.materialize()
            return True
        return False

    def release(self, slab) -> None:
        """The entry drops ``slab``: copy out every live row still in it."""
        for ref in self.refs.values():
            row = ref()
            if row is not None and row._slab is slab and row._dense is None:
                row.materialize()
        self.refs = {}
