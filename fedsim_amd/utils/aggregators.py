"""Aggregators — the drop-in boundary of the accelerated server path.

``SerialAggregator`` here is a duck-type-compatible replacement for the
reference's ``SerialAggregator`` (fedsim/utils/aggregators.py:11-144) whose
tensor-valued keys are reduced on the MI355X by libfedagg:

* ``add(key, tensor, weight)`` (aggregators.py:23-40) snapshots the client
  vector into a chunked HBM slab (H2D for CPU tensors, D2D for HIP tensors) and
  records ``fl32(weight)``; the running weight is the same Python sum
  ``cur_w + weight`` as the reference (so ``weight=None`` raises the same
  TypeError).  Full slabs are reduced by the exact-mode kernel into an fp32
  accumulator in arrival order.
* ``get`` / ``pop`` (aggregators.py:42-60, 104-122) reduce the pending rows and,
  when the weight is non-zero, divide by ``fl32(W)`` inside the same kernel
  pass.  The result is bit-identical to the reference CPU aggregation and is
  returned on the device the values came from (CPU in, CPU out).
* ``get_sum`` / ``get_weight`` / ``keys`` / ``items`` / ``pop_all`` /
  ``__contains__`` keep the reference semantics; a missing key raises
  ``Exception(f"{key} is not in the aggregator")``.

Python numbers and 0-dim tensors (the per-split scalar metrics that
serial_aggregation adds, training/utils.py:47-51) stay on the host with the
reference's own arithmetic.  N-d tensors must be float32: there is no CPU
fallback for them — without a HIP device / libfedagg the add raises.
"""
from __future__ import annotations

import os
from collections import deque
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from .dict_ops import apply_on_dict

__all__ = ["SerialAggregator", "DeviceAggregator", "AppendixAggregator"]

_DEFAULT_SLAB_BYTES = int(os.environ.get("FEDSIM_AMD_SLAB_BYTES", 16 << 30))
_DEFAULT_MAX_ROWS = int(os.environ.get("FEDSIM_AMD_MAX_ROWS", 4096))
_ROW_ALIGN = 64  # fp32 elements: 256-B aligned slab rows


def _hip_device(value: torch.Tensor, device) -> torch.device:
    if device is not None:
        return torch.device(device)
    if value.device.type == "cuda":
        return value.device
    if not torch.cuda.is_available():
        raise RuntimeError(
            "fedsim_amd.SerialAggregator reduces tensors on a HIP device, but none is "
            "available (no CPU fallback by design)"
        )
    return torch.device("cuda", torch.cuda.current_device())


class _DeviceEntry(object):
    """One tensor-valued key: fp32 running sum in HBM + pending client rows."""

    __slots__ = ("shape", "P", "ldx", "out_device", "dev", "acc", "cur_w", "chunks",
                 "rows_total", "n_pending", "pending_w", "max_rows", "flags")

    def __init__(self, value: torch.Tensor, dev: torch.device, slab_bytes: int,
                 max_rows: int, flags: int):
        self.shape = tuple(value.shape)
        self.P = value.numel()
        self.ldx = (self.P + _ROW_ALIGN - 1) // _ROW_ALIGN * _ROW_ALIGN
        self.out_device = value.device
        self.dev = dev
        self.acc: Optional[torch.Tensor] = None
        self.cur_w = 0
        self.chunks: List[torch.Tensor] = []
        self.rows_total = 0
        self.n_pending = 0
        self.pending_w: List[float] = []
        row_bytes = 4 * max(self.ldx, 1)
        self.max_rows = max(1, min(max_rows, slab_bytes // row_bytes))
        self.flags = flags

    # -- slab management ---------------------------------------------------
    def _row(self, i: int) -> torch.Tensor:
        for ch in self.chunks:
            if i < ch.shape[0]:
                return ch[i]
            i -= ch.shape[0]
        raise IndexError(i)

    def _grow(self) -> None:
        n = min(max(8, self.rows_total), self.max_rows - self.rows_total)
        self.chunks.append(torch.empty((n, self.ldx), dtype=torch.float32, device=self.dev))
        self.rows_total += n

    # -- reference semantics -------------------------------------------------
    def add(self, value: torch.Tensor, weight) -> None:
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        if tuple(value.shape) != self.shape:
            raise ValueError(
                f"tensor of shape {tuple(value.shape)} added to a key aggregating {self.shape}"
            )
        if value.dtype != torch.float32:
            raise TypeError(f"device aggregation supports float32 tensors, got {value.dtype}")
        w32 = float(np.float32(weight))
        if self.n_pending == self.max_rows:
            self._flush(final_W=None)
        if self.n_pending == self.rows_total:
            self._grow()
        dst = self._row(self.n_pending)[: self.P]
        src = value.detach().reshape(-1)
        # Snapshot now (the reference computes value * weight at add time).
        # Pinned CPU sources are copied synchronously so the caller may reuse them.
        dst.copy_(src, non_blocking=False)
        self.pending_w.append(w32)
        self.n_pending += 1
        self.cur_w = new_w

    def _flush(self, final_W) -> None:
        """Reduce pending rows into acc; divide by fl32(final_W) if given."""
        n = self.n_pending
        if n == 0:
            if final_W is not None and self.acc is not None:
                ops.finalize(self.acc, final_W, out=self.acc)
            return
        if self.acc is None:
            self.acc = torch.empty(self.P, dtype=torch.float32, device=self.dev)
            acc_in = None
        else:
            acc_in = self.acc
        rows = [self._row(i)[: self.P] for i in range(n)]
        w32 = torch.tensor(self.pending_w, dtype=torch.float32).pin_memory()
        w32 = w32.to(self.dev, non_blocking=True)
        table = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64).pin_memory()
        table = table.to(self.dev, non_blocking=True)
        ops.reduce_rows(rows, w32, self.acc, acc_in=acc_in, W=final_W, flags=self.flags,
                        table=table)
        self.n_pending = 0
        self.pending_w = []

    def _weighted(self) -> bool:
        return not (self.cur_w is None or self.cur_w == 0)

    def _deliver(self, t: torch.Tensor) -> torch.Tensor:
        t = t.view(self.shape)
        if self.out_device != t.device:
            t = t.to(self.out_device)  # D2H (or peer) copy; synchronises for CPU
        return t

    def get(self) -> torch.Tensor:
        self._flush(final_W=None)
        if not self._weighted():
            return self._deliver(self.acc.clone())
        return self._deliver(ops.finalize(self.acc, self.cur_w))

    def get_sum(self) -> torch.Tensor:
        self._flush(final_W=None)
        return self._deliver(self.acc.clone())

    def pop(self, on_device: bool = False) -> torch.Tensor:
        self._flush(final_W=self.cur_w if self._weighted() else None)
        out = self.acc.view(self.shape) if on_device else self._deliver(self.acc)
        self.chunks = []
        self.acc = None
        return out


class SerialAggregator(object):
    """Device-backed drop-in for the reference SerialAggregator
    (fedsim/utils/aggregators.py:11-144).

    Args:
        device: HIP device for tensor keys (default: the tensor's own device if
            it is a HIP tensor, else the current HIP device).
        slab_bytes: HBM budget for pending client rows per key; when full, the
            rows are reduced into the accumulator (order is preserved).
        max_rows: cap on pending rows per key.
        flags: libfedagg tuning flags (see include/fedagg.h).
    """

    def __init__(self, device=None, slab_bytes: int = _DEFAULT_SLAB_BYTES,
                 max_rows: int = _DEFAULT_MAX_ROWS, flags: int = 0) -> None:
        self._members: Dict = dict()
        self._device = device
        self._slab_bytes = slab_bytes
        self._max_rows = max_rows
        self._flags = flags

    @staticmethod
    def _is_device_value(value) -> bool:
        return isinstance(value, torch.Tensor) and value.dim() > 0

    def add(self, key, value, weight=None):
        entry = self._members.get(key)
        if isinstance(entry, _DeviceEntry):
            if not self._is_device_value(value):
                raise TypeError(f"key {key!r} aggregates tensors; got {type(value).__name__}")
            entry.add(value, weight)
            return
        if entry is None and self._is_device_value(value):
            dev = _hip_device(value, self._device)
            entry = _DeviceEntry(value, dev, self._slab_bytes, self._max_rows, self._flags)
            entry.add(value, weight)
            self._members[key] = entry
            return
        if entry is not None and self._is_device_value(value):
            raise TypeError(f"key {key!r} aggregates scalars; got an N-d tensor")
        # host path: the reference's own arithmetic (aggregators.py:17-40)
        new_v, new_w = (value, None) if weight is None else (value * weight, weight)
        sum_v, cur_w = self._members.get(key, (0, 0))
        if (sum_v is None) or (new_v is None):
            self._members[key] = (sum_v + new_v, None)
        else:
            self._members[key] = (sum_v + new_v, cur_w + new_w)

    def _entry(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        return self._members[key]

    def get(self, key):
        e = self._entry(key)
        if isinstance(e, _DeviceEntry):
            return e.get()
        v, w = e
        if w is None or w == 0:
            return v
        return v / w

    def get_sum(self, key):
        e = self._entry(key)
        if isinstance(e, _DeviceEntry):
            return e.get_sum()
        return e[0]

    def get_weight(self, key):
        e = self._entry(key)
        if isinstance(e, _DeviceEntry):
            return e.cur_w
        return e[1]

    def keys(self):
        return self._members.keys()

    def pop(self, key):
        e = self._entry(key)
        del self._members[key]
        if isinstance(e, _DeviceEntry):
            return e.pop()
        v, w = e
        if w is None or w == 0:
            return v
        return v / w

    def pop_device(self, key):
        """``pop`` that leaves a tensor result in HBM (no D2H), for the fused
        server step (not part of the reference API)."""
        e = self._entry(key)
        if not isinstance(e, _DeviceEntry):
            return self.pop(key)
        del self._members[key]
        return e.pop(on_device=True)

    def items(self):
        for key in self._members.keys():
            yield key, self.get(key)

    def pop_all(self):
        return {key: self.pop(key) for key in list(self._members.keys())}

    def __contains__(self, key):
        return key in self._members


DeviceAggregator = SerialAggregator


class AppendixAggregator(object):
    """Windowed history mean (reference: fedsim/utils/aggregators.py:147-318).

    Host-only; used by the round loop for score history, not on the
    accelerated path."""

    def __init__(self, max_deque_lenght=None) -> None:
        self._members = dict()
        self.max_deque_lenght = max_deque_lenght

    def append(self, key, value, weight=1, step=0):
        if key not in self._members:
            self._members[key] = tuple(deque(maxlen=self.max_deque_lenght) for _ in range(3))
        list_v, list_w, list_s = self._members[key]
        list_v.append(value)
        list_w.append(weight)
        list_s.append(step)

    def append_all(self, entry_dict, weight=1, step=0):
        apply_on_dict(entry_dict, self.append, weight=weight, step=step)

    def _check(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")

    def get(self, key, k=None):
        self._check(key)
        list_v, list_w, _ = (list(x) for x in self._members[key])
        n = len(list_v) if k is None else min(k, len(list_v))
        vs, ws = list_v[len(list_v) - n:], list_w[len(list_w) - n:]
        return sum(v * w for v, w in zip(vs, ws)) / sum(ws)

    def get_values(self, key):
        self._check(key)
        return self._members[key][0]

    def get_weights(self, key):
        self._check(key)
        return self._members[key][1]

    def get_steps(self, key):
        self._check(key)
        return self._members[key][2]

    def keys(self):
        return self._members.keys()

    def pop(self, key):
        self._check(key)
        list_v, list_w, _ = self._members.pop(key)
        return sum(v * w for v, w in zip(list_v, list_w)) / sum(list_w)

    def items(self):
        for key in self._members.keys():
            yield key, self.get(key)

    def pop_all(self):
        return {key: self.pop(key) for key in list(self._members.keys())}

    def __contains__(self, key):
        return key in self._members
