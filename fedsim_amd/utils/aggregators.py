"""Aggregators — the drop-in boundary of the accelerated server path.

``SerialAggregator`` here is a duck-type-compatible replacement for the
reference's ``SerialAggregator`` (fedsim/utils/aggregators.py:11-144) whose
tensor-valued keys are reduced on the MI355X by libfedagg:

* ``add(key, tensor, weight)`` (aggregators.py:23-40) snapshots the client
  vector into a column-blocked HBM ring slab and records ``fl32(weight)``; the
  running weight is the same Python sum ``cur_w + weight`` as the reference (so
  ``weight=None`` raises the same TypeError).  HIP-resident vectors are packed
  by a copy kernel on the compute stream; host vectors are snapshotted into a
  pinned staging ring and packed on a separate copy stream (the pack kernel
  reading the slot in place over PCIe, or a DMA: ``_HOST_PACK``), overlapping
  the reductions.
* Pending rows are reduced by the exact-mode kernel into an fp32 accumulator in
  arrival order whenever the ring needs room, and at ``get`` / ``pop``
  (aggregators.py:42-60, 104-122), where the divide by ``fl32(W)`` is fused
  into the same kernel pass.  Results are bit-identical to the reference CPU
  aggregation and come back on the device the values came from (CPU in, CPU
  out).
* ``get_sum`` / ``get_weight`` / ``keys`` / ``items`` / ``pop_all`` /
  ``__contains__`` keep the reference semantics; a missing key raises
  ``Exception(f"{key} is not in the aggregator")``.

Every other value keeps the reference's own arithmetic, exactly as
aggregators.py:17-40 writes it (``sum_v + value * weight`` with torch's type
promotion, on the value's own device):

* Python numbers and 0-dim tensors (the per-split scalar metrics that
  serial_aggregation adds, training/utils.py:47-51);
* N-d tensors of any other dtype (fp64, bf16 / fp16, integer, bool): an fp64
  or bf16 model's parameters, a plugin's per-class counts.  Their ``v / w``
  at ``get`` / ``pop`` is ATen CPU's true division -- in f64 for an fp64 sum
  (fedagg_finalize_f64), in f32 for the others (fedagg_finalize_f32), the
  rounding ATen's CPU kernel gives and torch's own HIP kernel (a multiply by
  the reciprocal) does not -- so HIP-resident keys match the reference CPU
  aggregation bit for bit;
* a tensor key that stops fitting the kernel -- a value of another dtype or
  shape, a non-real weight, a scalar added to it -- leaves it: its exact
  running sum so far continues under the reference's arithmetic, so torch's
  promotion (fp32 sum + fp64 value -> fp64) and broadcasting apply as in the
  reference.

fp32 N-d tensors have no CPU fallback: without a HIP device / libfedagg the
add raises.
"""
from __future__ import annotations

import functools
import os
import struct
from collections import deque
import threading
from concurrent.futures import Future, ThreadPoolExecutor
from concurrent.futures import wait as _wait_futures
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from .dict_ops import apply_on_dict
from .slab_rows import RowRefs, SlabRow

__all__ = ["SerialAggregator", "DeviceAggregator", "AppendixAggregator"]

_ENV_SLAB_BYTES = os.environ.get("FEDSIM_AMD_SLAB_BYTES")
_DEFAULT_SLAB_BYTES = int(_ENV_SLAB_BYTES) if _ENV_SLAB_BYTES else None
_SLAB_CAP = 64 << 30  # per key; a quarter of HBM at most (288 GB on MI355X)


def _slab_budget(dev: torch.device, requested: Optional[int]) -> int:
    """HBM budget of one key's ring.  Each drain re-reads and re-writes the
    4P-byte accumulator, so a long ring keeps that overhead at ~1 % (SURVEY
    §8d): default min(64 GiB, total HBM / 4)."""
    if requested is not None:
        return requested
    total = torch.cuda.get_device_properties(dev).total_memory
    return min(_SLAB_CAP, total // 4)
_DEFAULT_MAX_ROWS = int(os.environ.get("FEDSIM_AMD_MAX_ROWS", 4096))
_F32 = struct.Struct("f")


def _fl32(x) -> float:
    """fl32(x) as a Python float: ATen's rounding of a Python scalar weight
    (round to nearest even), the same as float(np.float32(x))."""
    return _F32.unpack(_F32.pack(x))[0]
# Staging slots of the ingest ring (pinned host + device buffers of one
# vector each): five keep a DMA, a pack kernel and the next staging copy in
# flight together -- against three, config 2 K=1000 host rounds 100.9 vs
# 106.4 ms, 16 MB host->host rounds 47.0-47.1 vs 45.0-45.9 GB/s, 100 MB
# +0.5 % (profiles/r06w/ab_staging_slots.jsonl).
_STAGING_SLOTS = 5

# How the ingest worker copies a handed-over pageable vector into pinned
# staging: "auto", "torch" (torch's multi-threaded copy_) or "memmove<N>" (N
# threads of ctypes memmove).  Interleaved on one box (tools/ab_staging.py,
# profiles/r06o/): below 32 MB torch's copy_ wins (a K=10 x 4.3 MB round
# 1.39-1.41 ms against 1.92-1.98 for four memmoves, 2.0-2.3 for one); at
# 100 MB four memmoves keep the round at the link (53.2-53.4 GB/s against
# 43-46 for torch's copy_, whose 16 threads take the host memory bandwidth
# the concurrent DMA reads from).  At 100 MB six threads keep the copy ahead
# of the 53 GB/s DMA with headroom: over two boxes (profiles/r06w/
# ab_staging_threads*.jsonl) the pageable round's median is 53.1 GB/s with
# six threads against 49.5 with four (nine rounds each; eight: no better).
# "auto" takes torch's copy below 32 MB and six threads from 32 MB.
_STAGE_COPY = os.environ.get("FEDSIM_AMD_STAGE_COPY", "auto")
# How a page-locked host vector (the caller's, or the staging slot) reaches
# its slab row: "zero_copy", the pack kernel reading it in place over PCIe
# (fedagg_pack_row_f32 on a mapped host pointer: no DMA to issue), "dma", a
# DMA into a device slot and then the HBM pack (rounds 1-5), or "auto".
# Interleaved on one box (tools/ab_host_pack.py, profiles/r06w/): for
# vectors staged from pageable memory the kernel wins below 64 MB (config 1
# rounds 0.45 vs 0.52 ms, config 2 K=1000 113 vs 124 ms, 4.3 / 32 MB
# host->host rounds 36.1 / 48.4 vs 34.3 / 44.4 GB/s) and the two are within
# noise at 100 MB; for the caller's own pinned vectors, whose put waits for
# the copy, the DMA engine wins (4.3 / 32 / 100 MB: 36.3 / 51.2 / 52.5 vs
# 31.9 / 47.7 / 50.9 GB/s).  "auto" takes the kernel for staged vectors
# below 2 MB, alternates the two from 2 MB (_MIXED_MIN) and takes the DMA
# from 64 MB and for the caller's own pinned vectors.
_HOST_PACK = os.environ.get("FEDSIM_AMD_HOST_PACK", "auto")
_ZERO_COPY_MAX = 64 << 20
# From 2 MB "auto" alternates the two routes per staged vector, so the DMA
# engine and the pack kernel share the link (profiles/r06w/
# ab_host_pack_mixed.jsonl, against the kernel alone: config 2 K=1000 host
# rounds 104.4 vs 112.0 ms, 4.3 MB host->host rounds 39.9 / 40.4 vs 36.3 /
# 35.8 GB/s pinned / pageable; at 0.8 MB, config 1, it loses: 0.38 vs 0.34 ms).
_MIXED_MIN = 2 << 20
# The ingest ring's DMAs and packs on two streams (the DMA engine does not
# idle while a pack runs), and the caller's handed-over pinned vectors
# checked at the reduction instead of after each DMA (the worker does not
# idle between DMAs); "0" restores one stream and per-put waits (A/B).
_INGEST_OVERLAP = os.environ.get("FEDSIM_AMD_INGEST_OVERLAP", "1") == "1"
# The caller's own pinned vectors from this size on are DMA'd straight from
# its buffer, the put waiting for the DMA so the caller may reuse it; smaller
# ones are staged like pageable vectors (a pinned-to-pinned copy, then the
# put returns): profiles/r06N/plugin_round.jsonl had pinned rounds slower
# than pageable ones below 32 MB (config 1 0.48 vs 0.36 ms, config 2 K=10
# 1.46 vs 1.24 ms) and faster at 100 MB (53.0 vs 51.2 GB/s).
_PINNED_DIRECT_MIN = int(os.environ.get("FEDSIM_AMD_PINNED_DIRECT_MIN", 32 << 20))
_STAGE_SPLIT_MIN = 32 << 20
_stage_pool: Optional[ThreadPoolExecutor] = None


def _host_route(pinned: bool, nbytes: int, odd: bool = False):
    """(direct, dma) for a host vector of ``nbytes`` reaching its slab row:
    ``direct`` -- DMA'd straight from the caller's pinned buffer rather than
    staged (_PINNED_DIRECT_MIN); ``dma`` -- through a device slot and the HBM
    pack rather than the pack kernel reading the page-locked vector in place
    (_HOST_PACK, _ZERO_COPY_MAX).  "mixed" alternates the two for staged
    vectors (``odd``: every second one), so the DMA engine and the pack
    kernel share the link."""
    direct = pinned and nbytes >= _PINNED_DIRECT_MIN
    if _HOST_PACK == "dma":
        return direct, True
    if _HOST_PACK == "zero_copy":
        return direct, False
    if _HOST_PACK == "mixed":
        return direct, direct or nbytes >= _ZERO_COPY_MAX or odd
    return direct, direct or nbytes >= _ZERO_COPY_MAX or (nbytes >= _MIXED_MIN and odd)


def _staging_copy(dst: torch.Tensor, src: torch.Tensor) -> None:
    """dst.copy_(src) for a pinned fp32 slot and a source of its size, by
    _STAGE_COPY's method."""
    global _stage_pool
    how = _STAGE_COPY
    if how == "auto":
        how = "memmove6" if 4 * src.numel() >= _STAGE_SPLIT_MIN else "torch"
    if how == "torch" or not (src.is_contiguous() and src.dtype == torch.float32):
        dst.copy_(src)
        return
    import ctypes

    n = max(1, int(how[len("memmove"):] or 1))
    nbytes, d, s = 4 * src.numel(), dst.data_ptr(), src.data_ptr()
    if n == 1:
        ctypes.memmove(d, s, nbytes)
        return
    if _stage_pool is None or _stage_pool._max_workers < n - 1:
        _stage_pool = ThreadPoolExecutor(max_workers=n - 1, thread_name_prefix="fedsim-stage")
    step = (-(-nbytes // n) + 4095) & ~4095  # page-rounded, n * step >= nbytes
    futs = [_stage_pool.submit(ctypes.memmove, d + i * step, s + i * step,
                               min(step, nbytes - i * step))
            for i in range(1, n) if i * step < nbytes]
    ctypes.memmove(d, s, min(step, nbytes))
    for f in futs:
        f.result()


def to_host(t: torch.Tensor) -> torch.Tensor:
    """A HIP tensor delivered to the host in page-locked memory: one DMA at
    PCIe rate.  A pageable destination ran at 6.7 GB/s on the MI355X box
    (first-touch faults of fresh pages behind the runtime's staging), a
    pinned one at 56.8 GB/s (tools/probe_h2d.py, profiles/r06b/): for the
    25 M-parameter average, 15 ms against 1.8 ms.  The result is an ordinary
    CPU tensor (``is_pinned()`` is True); torch's host allocator recycles the
    block once it is freed."""
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return h


def _deliver_to(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """``t.to(device)`` with the D2H leg through pinned memory."""
    if t.device == device:
        return t
    if device.type == "cpu" and t.device.type == "cuda" and not t.requires_grad:
        return to_host(t)
    return t.to(device)


def _on_own_device(fn):
    """Run an entry method with the entry's GPU as the current device:
    libfedagg launches on the stream it is handed, and HIP launches go to the
    current device's queues (a key on cuda:1 used while cuda:0 is current,
    or one shard of a single-process multi-GPU key)."""
    @functools.wraps(fn)
    def on_device(self, *args, **kwargs):
        idx = getattr(self.dev, "index", None)
        if idx is None or torch.cuda.current_device() == idx:
            return fn(self, *args, **kwargs)
        with torch.cuda.device(idx):
            return fn(self, *args, **kwargs)
    return on_device


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


class _Ingest(object):
    """Staging ring + copy stream for host-resident client vectors.

    ``put`` snapshots the vector (pageable sources: a CPU copy into a pinned
    slot, which is the reference's clone; the caller may reuse its tensor as
    soon as add returns), DMAs it whole into a device slot with one 1-D copy on
    the copy stream, and scatters that into the slab row with the pack kernel
    on the same stream.  A 2-D DMA straight into the column-blocked row costs
    one descriptor per C-float segment: at C = 1024 (P < 8 M) that ran at
    2 GB/s, against PCIe's 55 for the whole vector.  A slot is reused only
    after its previous copies have completed.  One ring per device is shared
    by all aggregators (the round driver makes a new one every round).

    The puts run one at a time in submission order (the slots and the copy
    stream see one sequence).  ``put`` runs on the calling thread, after any
    queued asynchronous put: the snapshot is taken when add returns, as the
    reference's clone.  ``put_async`` runs on ONE worker thread and returns
    at once: for a host vector the client handed over (the
    round driver's borrowing aggregator, training/utils.py ``_handed_over``),
    the pageable-to-pinned copy and the DMA then run while the next client
    trains instead of between the two clients (tools/bench_host_rounds.py:
    0.2-1.5 ms per client on the critical path otherwise).  A handed-over
    vector changed in place (an in-place torch op: its version counter) from
    ``add`` until its copy has completed is caught and raised at the round's
    reduction: a staged vector's counter is checked before and after its copy
    into staging (a later change cannot alter the row); a pinned vector DMA'd
    straight from the caller's buffer is checked when the reduction waits for
    that DMA, so any change before then raises, as for a borrowed HBM row."""

    def __init__(self, dev: torch.device, nslots: int = _STAGING_SLOTS):
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev)  # DMAs into the device slots
        self.pack_stream = torch.cuda.Stream(device=dev)  # packs into the slab rows
        self.hbufs: List[Optional[torch.Tensor]] = [None] * nslots
        self.dbufs: List[Optional[torch.Tensor]] = [None] * nslots
        self.events: List[Optional[torch.cuda.Event]] = [None] * nslots
        self.i = 0
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="fedsim-ingest",
                                       initializer=torch.cuda.set_device, initargs=(dev,))
        self.lock = threading.Lock()
        self.last: Optional[Future] = None  # the latest asynchronous put

    def drain(self) -> None:
        """Every DMA and pack issued so far has completed."""
        self.stream.synchronize()
        self.pack_stream.synchronize()

    def put(self, src: torch.Tensor, Xb: torch.Tensor, r: int, wait_event=None):
        if self.last is not None:
            _wait_futures([self.last])  # its error, if any, is its entry's to raise
            self.last = None
        return self._put(src, Xb, r, wait_event, None)

    def put_async(self, src: torch.Tensor, Xb: torch.Tensor, r: int, wait_event=None) -> Future:
        """Future of put's event; ``src`` must not change until it resolves."""
        self.last = self.pool.submit(self._put, src, Xb, r, wait_event, src._version)
        return self.last

    @staticmethod
    def _slot(bufs, i, P, **kw):
        buf = bufs[i]
        if buf is None or buf.numel() < P:
            buf = torch.empty(max(P, 1), dtype=torch.float32, **kw)
            bufs[i] = buf
        return buf[:P]

    def _put(self, src, Xb, r, wait_event, version):
        with self.lock:
            return self._put_locked(src, Xb, r, wait_event, version)

    @staticmethod
    def _check_version(src, version):
        if version is not None and src._version != version:
            raise RuntimeError(
                "a host client tensor was modified in place after SerialAggregator.add(); "
                "an aggregator created with borrow=True copies it after add returns (use "
                "borrow=False to snapshot it at add time)")

    def _put_locked(self, src, Xb, r, wait_event, version):
        self._check_version(src, version)
        i = self.i % len(self.events)
        self.i += 1
        if self.events[i] is not None:
            self.events[i].synchronize()
        P = src.numel()
        direct, dma = _host_route(src.is_pinned(), 4 * P, odd=bool(self.i & 1))
        if direct:
            host = src  # DMA straight from the caller's pinned buffer
        else:
            host = self._slot(self.hbufs, i, P, pin_memory=True)
            # on the ingest worker too, while the next client trains: a
            # multi-threaded copy (_staging_copy; one memmove ran at 29 GB/s
            # from cold client memory, tools/probe_put.py, profiles/r06m/),
            # which meets the clients' training threads for tens of
            # microseconds per client
            _staging_copy(host, src)
            self._check_version(src, version)  # not changed while it was copied
        packed = host  # the pack kernel reads it in place over PCIe
        pack_stream = self.pack_stream if _INGEST_OVERLAP else self.stream
        if dma:
            # a DMA into a device slot, then the HBM pack -- on its own stream,
            # so the next vector's DMA does not queue behind this pack
            packed = self._slot(self.dbufs, i, P, device=self.dev)
            with torch.cuda.stream(self.stream):
                packed.copy_(host, non_blocking=True)
            if pack_stream is not self.stream:
                pack_stream.wait_stream(self.stream)
        if wait_event is not None:
            pack_stream.wait_event(wait_event)
        ops.pack_row(packed, Xb, r, stream=pack_stream)
        ev = torch.cuda.Event()
        ev.record(pack_stream)
        self.events[i] = ev
        if direct:
            if version is not None and _INGEST_OVERLAP:
                # handed over: the worker moves on to the next vector; the
                # entry waits for this copy and checks the version at the
                # reduction (_DeviceEntry._copies_issued), where a change
                # made in place before the round is reduced raises as for a
                # borrowed HBM row (utils/handover.py)
                return ev, (src, version, ev)
            # the snapshot is complete once the DMA is: the caller may reuse
            # its pinned buffer after add returns
            ev.synchronize()
            self._check_version(src, version)
        return ev


_INGESTS: Dict = {}

# Handed-over host vectors from this many floats (2 MB) on are staged by the
# ingest worker; smaller ones on the calling thread at add.  With the clients'
# training in the loop (tools/bench_host_rounds.py, profiles/r04i, r04k) the
# worker saves 2.5-3 ms per round at config 2 (4.3 MB vectors: receive 1.0-1.7
# vs 3.5-4.7 ms), while at config 1 (0.8 MB) its hand-off costs more at
# optimize than the copies it moves (receive + optimize 1.1-1.4 vs 1.0-1.2 ms).
_ASYNC_STAGE_MIN = 1 << 19


# Borrowed client tensors after the reduction that read them was enqueued:
# kept alive until its completion event, so their memory cannot be reused by
# another stream while the kernel still reads it.  This replaces one
# ``record_stream`` per row (≈1 µs of host time each: ≈1 ms for a
# 1000-client round) with one list entry per reduction; completed entries
# are dropped whenever a round adds or drains rows.
_KEEPALIVE: deque = deque()


def _keep_until(event, tensors) -> None:
    _KEEPALIVE.append((event, tensors))
    _prune_keepalive()


def _prune_keepalive(wait: bool = False) -> None:
    """Drop the entries whose reduction has run (``wait``: all of them, once
    they have run -- the round driver calls this when training returns, so
    the last round's client tensors are not held after it)."""
    while _KEEPALIVE and (wait or _KEEPALIVE[0][0].query()):
        ev, _ = _KEEPALIVE.popleft()
        if wait:
            ev.synchronize()


_PRUNE_EVERY = 32  # adds between two completion queries while entries are pending
_prune_tick = 0


def _prune_keepalive_at_add() -> None:
    """The prune an ``add`` runs: one event query per _PRUNE_EVERY adds (the
    last round's reduction may still be running through the first adds of
    the next round; a query per add is ≈1 µs of host time per client)."""
    global _prune_tick
    _prune_tick += 1
    if _prune_tick >= _PRUNE_EVERY:
        _prune_tick = 0
        _prune_keepalive()


def release_borrowed() -> None:
    """Wait for every reduction still reading borrowed client tensors and
    release them."""
    _prune_keepalive(wait=True)


def _ingest_for(dev: torch.device) -> _Ingest:
    ing = _INGESTS.get(dev)
    if ing is None:
        ing = _INGESTS[dev] = _Ingest(dev)
    return ing


class _Like(object):
    """Shape / size / device of a key's vectors before any value arrives."""

    def __init__(self, shape, device):
        self.shape = shape
        self.device = device
        self._n = 1
        for d in shape:
            self._n *= d

    def numel(self):
        return self._n


class _Options(object):
    __slots__ = ("device", "slab_bytes", "max_rows", "flags", "expected_rows", "block_cols",
                 "borrow", "fast", "borrow_host")

    def __init__(self, device, slab_bytes, max_rows, flags, expected_rows, block_cols,
                 borrow=False, fast=False, borrow_host=False):
        self.device = device
        self.slab_bytes = slab_bytes
        self.max_rows = max_rows
        self.flags = flags
        self.expected_rows = expected_rows
        self.block_cols = block_cols
        self.borrow = borrow
        self.fast = fast
        self.borrow_host = borrow_host


class _TensorEntry(object):
    """What SerialAggregator needs from the state of one tensor-valued key:
    ``add(value, weight)``, ``get()``, ``get_sum()``, ``pop(on_device)``,
    ``pop_step(step)``, the running Python weight ``cur_w`` and the device
    ``dev`` the reduction runs on.  _DeviceEntry is the one-GPU key;
    fedsim_amd.sharding._ShardEntry spreads a key's columns over the ranks of
    a process group."""

    cur_w = 0
    dev = None
    shape = ()
    out_device = None  # the first value's device (None: not tracked)

    def takes(self, value, weight) -> bool:
        """Whether this entry adds (value, weight) itself; otherwise the key
        leaves it for the reference's arithmetic (SerialAggregator.add).  A
        value on another device than the key's first value is left to that
        arithmetic too, where ``sum_v + new_v`` raises as in the reference
        (aggregators.py:38,40) and the key stays as it was: the rule is
        relative to the delivery device, not the compute device (host values
        into HIP shards are one device)."""
        return (_kernel_value(value, weight) and tuple(value.shape) == self.shape
                and (self.out_device is None or value.device == self.out_device))


class _DeviceEntry(_TensorEntry):
    """One tensor-valued key: fp32 running sum in HBM + a ring of pending
    client rows in a column-blocked slab [ceil(P/C), R, C] (include/fedagg.h).
    ``out_device``: where get / pop deliver (default: the first value's
    device, as the reference's tensors stay where they were added)."""

    def __init__(self, value: torch.Tensor, dev: torch.device, opts: _Options, agg,
                 out_device: Optional[torch.device] = None):
        self.shape = tuple(value.shape)
        self.P = value.numel()
        self.out_device = value.device if out_device is None else out_device
        self.dev = dev
        self.C = opts.block_cols or ops.choose_block_cols(self.P)
        self.nblk = (self.P + self.C - 1) // self.C
        row_bytes = 4 * max(1, self.nblk) * self.C
        budget = _slab_budget(dev, opts.slab_bytes)
        self.Rmax = max(2, min(opts.max_rows, budget // row_bytes))
        # borrowed rows: HBM-resident client tensors reduced in place (no
        # snapshot copy); at most Bmax are held before they are drained
        self.borrow = opts.borrow
        self.borrow_host = opts.borrow_host
        self.Bmax = max(1, min(opts.max_rows, budget // max(4, 4 * self.P)))
        self.borrowed: List = []
        self.borrowed_ptrs: List[int] = []  # their data pointers (the row table)
        # grow the ring without draining it (chained partial sums, _grow)
        self.keep_pending = False
        self.R = 0
        self.slab: Optional[torch.Tensor] = None
        self.hint = opts.expected_rows
        self.flags = ops.default_flags(self.C) if opts.flags is None else opts.flags
        if opts.fast:
            self.flags |= ops.FEDAGG_FAST
        self.agg = agg
        self.head = 0
        self.tail = 0
        self.n_pending = 0
        self.pending_w: List[float] = []
        self.acc: Optional[torch.Tensor] = None
        self.cur_w = 0
        self.rows = RowRefs()        # SlabRows handed out by reserve()
        self.copy_event = None       # last host DMA into the slab (copy stream)
        self.staging: List[Future] = []  # ingest-worker puts not yet checked
        self.failed: Optional[BaseException] = None  # a failed put: the ring is incomplete
        self.last_flush_event = None  # last reduction reading the slab (compute stream)
        self.wait_before_copy = None

    # -- ring management -----------------------------------------------------
    def _copies_issued(self) -> None:
        """Host rows still being staged by the ingest worker have been issued
        on its copy stream (copy_event is then their event).  Every pending
        put is checked, not only the last: the first failure (a tensor
        modified in place, an allocation or HIP error) is raised here, so a
        row that was never written cannot reach a reduction."""
        if self.failed is not None:  # a row was never written: every later use refuses
            raise self.failed
        if self.staging:
            futs, self.staging = self.staging, []
            _wait_futures(futs)
            for f in futs:
                err = f.exception()
                if err is None and isinstance(f.result(), tuple):
                    # a handed-over pinned vector DMA'd straight from the
                    # caller's buffer: unchanged until its copy completed?
                    src, version, done = f.result()[1]
                    done.synchronize()
                    try:
                        _Ingest._check_version(src, version)
                    except RuntimeError as e:
                        err = e
                if err is not None:
                    self.copy_event = None
                    self.failed = err
                    raise self.failed
        if isinstance(self.copy_event, Future):
            res = self.copy_event.result()
            self.copy_event = res[0] if isinstance(res, tuple) else res

    def _alloc(self, rows: int) -> None:
        self._copies_issued()
        if self.slab is not None:
            self.rows.release(self.slab)
        self.slab = torch.empty((self.nblk, rows, self.C), dtype=torch.float32, device=self.dev)
        self.R = rows
        self.head = self.tail = 0
        # a recycled block may still be read by an earlier reduction: the first
        # host DMA into the new slab waits for the latest one
        self.wait_before_copy = self.last_flush_event

    def _grow(self, rows: int) -> None:
        """A larger ring that keeps the pending rows, in arrival order, as its
        first rows (two D2D copies on the compute stream) instead of draining
        them: a chained partial sum (client-sharded rounds) must see every row
        of this rank still pending when the chain reaches it."""
        self._copies_issued()
        cur = torch.cuda.current_stream(self.dev)
        if self.copy_event is not None:
            cur.wait_event(self.copy_event)
            self.copy_event = None
        old, n, t = self.slab, self.n_pending, self.tail
        new = torch.empty((self.nblk, rows, self.C), dtype=torch.float32, device=self.dev)
        first = min(n, self.R - t)
        new[:, :first].copy_(old[:, t:t + first])
        if n > first:
            new[:, first:n].copy_(old[:, :n - first])
        self.rows.release(old)
        self.slab, self.R, self.tail, self.head = new, rows, 0, n % rows
        # host DMAs into the new ring (copy stream) start after everything the
        # compute stream has queued: its block may be recycled memory
        ev = torch.cuda.Event()
        ev.record(cur)
        self.wait_before_copy = ev

    def _make_room(self) -> None:
        if self.slab is None:
            first = self.hint if self.hint else 8
            self._alloc(min(self.Rmax, max(1, first)))
            return
        if self.R < self.Rmax:
            if self.n_pending == self.R:
                if self.keep_pending:
                    self._grow(min(self.Rmax, 2 * self.R))
                    return
                self._flush(final_W=None)
                self._alloc(min(self.Rmax, 2 * self.R))
        elif self.n_pending >= max(1, self.Rmax // 2):
            # double buffering: drain one half while the other half fills
            self._flush(final_W=None)

    def _claim(self, r: int) -> None:
        """Row r is about to be written: a live SlabRow still showing it is
        copied out first, and the next host DMA waits for that copy."""
        if self.rows.claim(r, self.slab):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self.wait_before_copy = ev

    @_on_own_device
    def reserve(self) -> SlabRow:
        """The next ring row, as a SlabRow a client can vectorize its model
        into (slab_rows.py); ``add`` of that row commits it in place."""
        if self.borrowed:
            self._flush(final_W=None)  # earlier borrowed rows first: arrival order
        self._make_room()
        r = self.head
        self._claim(r)
        row = SlabRow(self, self.slab, r, self.P)
        self.rows.track(row)
        return row

    @_on_own_device
    def release(self) -> None:
        """Drop the slab; SlabRows still alive keep a copy of their row.  A
        failed staging put is not raised again here (add and the reductions
        raise it): a cleanup must not hide the first error.  The copy stream
        is drained instead, so no DMA still writes into the freed slab."""
        try:
            self._copies_issued()
        except BaseException:  # noqa: BLE001 -- the entry's own calls raise it
            self.copy_event = None
            self.agg._ingest(self.dev).drain()
        if self.copy_event is not None:  # the slab is read by the copy stream until then
            self.copy_event.synchronize()
            self.copy_event = None
        if self.slab is not None:
            self.rows.release(self.slab)
        self.slab = None

    # -- reference semantics -------------------------------------------------
    @_on_own_device
    def add(self, value: torch.Tensor, weight) -> None:
        if _KEEPALIVE:  # an earlier round's borrowed rows, once it has run
            _prune_keepalive_at_add()
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        if value.shape != self.shape:
            raise ValueError(
                f"tensor of shape {tuple(value.shape)} added to a key aggregating {self.shape}"
            )
        if value.dtype != torch.float32:
            raise TypeError(f"device aggregation supports float32 tensors, got {value.dtype}")
        w32 = _fl32(weight)
        # the common case (a detached flat vector from vectorize_module) is
        # taken as is: detach / reshape allocate a new tensor object each,
        # a few us per client on the host
        src = value.detach() if value.requires_grad else value
        if isinstance(src, SlabRow):
            if (src._entry is self and src.in_slab and src._slab is self.slab
                    and src._row == self.head and not src._committed):
                # the client wrote its vector into the row reserved for it:
                # commit in place (vectorize_module(..., out=reserve()))
                if self.borrowed:
                    self._flush(final_W=None)
                src._committed = True
                self.head = (self.head + 1) % self.R
                self.n_pending += 1
                self.pending_w.append(w32)
                self.cur_w = new_w
                return
            src = src.materialize()  # another entry's row, or a stale one
        if src.dim() != 1:
            src = src.reshape(-1)
        if self.borrow and self._borrowable(src):
            if self.n_pending:
                self._flush(final_W=None)  # earlier slab rows first: arrival order
            elif len(self.borrowed) >= self.Bmax:
                self._flush(final_W=None)
            self.borrowed.append((src, src._version))
            self.borrowed_ptrs.append(src.data_ptr())
            self.pending_w.append(w32)
            self.cur_w = new_w
            return
        if self.borrowed:
            self._flush(final_W=None)
        self._make_room()
        r = self.head
        self._claim(r)
        if src.device.type == "cuda":
            if src.device != self.dev:
                src = src.to(self.dev)
            ops.pack_row(src.contiguous(), self.slab, r)  # D2D on the compute stream
        elif self.borrow_host and src.is_contiguous() and src.numel() >= _ASYNC_STAGE_MIN:
            # handed over (serial_aggregation clones otherwise): copied while
            # the next client trains
            self.copy_event = self.agg._ingest(self.dev).put_async(
                src, self.slab, r, wait_event=self.wait_before_copy)
            self.staging.append(self.copy_event)
            self.wait_before_copy = None
        else:
            self.copy_event = self.agg._ingest(self.dev).put(
                src.contiguous(), self.slab, r, wait_event=self.wait_before_copy)
            self.wait_before_copy = None
        self.head = (r + 1) % self.R
        self.n_pending += 1
        self.pending_w.append(w32)
        self.cur_w = new_w

    def _borrowable(self, src: torch.Tensor) -> bool:
        return (src.device == self.dev and src.is_contiguous() and src.data_ptr() % 16 == 0
                and src.numel() > 0)

    def _flush_borrowed(self, final_W, step: Optional[ops.ServerStep] = None) -> None:
        """Reduce the borrowed rows in place (pointer table, arrival order)."""
        rows = []
        for t, version in self.borrowed:
            if t._version != version:
                raise RuntimeError(
                    "a client tensor was modified in place after SerialAggregator.add(); "
                    "an aggregator created with borrow=True reads it when the round is "
                    "reduced (use borrow=False to snapshot it at add time)")
            rows.append(t)
        cur = torch.cuda.current_stream(self.dev)
        w32 = torch.tensor(self.pending_w, dtype=torch.float32, pin_memory=True)
        w32 = w32.to(self.dev, non_blocking=True)
        table = ops.row_table_from_ptrs(self.borrowed_ptrs, self.dev)
        # every row passed _borrowable at add: skip the per-row checks
        if step is not None:
            ops.reduce_rows_step(rows, w32, step, acc_in=self.acc, W=final_W, table=table,
                                 checked=True, flags=self.flags & ops.FEDAGG_FAST)
        else:
            acc_in = self.acc
            if self.acc is None:
                self.acc = torch.empty(self.P, dtype=torch.float32, device=self.dev)
            ops.reduce_rows(rows, w32, self.acc, acc_in=acc_in, W=final_W,
                            flags=ops.FEDAGG_NT | (self.flags & ops.FEDAGG_FAST), table=table,
                            checked=True)
        # the caller's allocations may belong to another stream: they stay
        # alive until this reduction has run (instead of a record_stream each)
        ev = torch.cuda.Event()
        ev.record(cur)
        _keep_until(ev, rows)
        self.borrowed = []
        self.borrowed_ptrs = []
        self.pending_w = []

    def _flush(self, final_W, step: Optional[ops.ServerStep] = None) -> None:
        """Reduce the pending rows into acc (arrival order); divide by
        fl32(final_W) in the same pass if given.  With ``step``, the last
        segment's pass also runs the server step on the result instead of
        storing it (pop + optimize in one pass; needs pending rows)."""
        if self.borrowed:
            self._flush_borrowed(final_W, step)
            return
        n = self.n_pending
        cur = torch.cuda.current_stream(self.dev)
        if n == 0:
            if final_W is not None and self.acc is not None:
                ops.finalize(self.acc, final_W, out=self.acc)
            return
        self._copies_issued()
        if self.copy_event is not None:
            cur.wait_event(self.copy_event)
            self.copy_event = None
        acc_in = self.acc
        w32 = torch.tensor(self.pending_w, dtype=torch.float32, pin_memory=True)
        w32 = w32.to(self.dev, non_blocking=True)
        first = self.R - self.tail
        segs = [(self.tail, n)] if n <= first else [(self.tail, first), (0, n - first)]
        off = 0
        for i, (r0, cnt) in enumerate(segs):
            last = i == len(segs) - 1
            if last and step is not None:
                ops.reduce_blocked_step(self.slab, w32[off:off + cnt], step, B=cnt,
                                        acc_in=acc_in, W=final_W, r0=r0,
                                        flags=self.flags & ops.FEDAGG_FAST)
            else:
                if self.acc is None:
                    self.acc = torch.empty(self.P, dtype=torch.float32, device=self.dev)
                ops.reduce_blocked(self.slab, w32[off:off + cnt], self.acc, B=cnt,
                                   acc_in=acc_in, W=final_W if last else None,
                                   flags=self.flags, r0=r0)
                acc_in = self.acc
            off += cnt
        ev = torch.cuda.Event()
        ev.record(cur)
        self.last_flush_event = ev
        self.wait_before_copy = ev
        self.tail = (self.tail + n) % self.R
        self.n_pending = 0
        self.pending_w = []

    def _weighted(self) -> bool:
        return not (self.cur_w is None or self.cur_w == 0)

    def _deliver(self, t: torch.Tensor) -> torch.Tensor:
        return _deliver_to(t.view(self.shape), self.out_device)  # D2H: pinned, synchronised

    @_on_own_device
    def get(self) -> torch.Tensor:
        self._flush(final_W=None)
        if not self._weighted():
            return self._deliver(self.acc.clone())
        return self._deliver(ops.finalize(self.acc, self.cur_w))

    @_on_own_device
    def get_sum(self) -> torch.Tensor:
        self._flush(final_W=None)
        return self._deliver(self.acc.clone())

    @_on_own_device
    def pop(self, on_device: bool = False) -> torch.Tensor:
        self._flush(final_W=self.cur_w if self._weighted() else None)
        out = self.acc.view(self.shape) if on_device else self._deliver(self.acc)
        self.release()
        self.acc = None
        return out

    def chainable(self) -> bool:
        """Whether ``partial`` can still continue another rank's sum: no row
        has been drained into the accumulator from +0 yet."""
        return self.acc is None

    @_on_own_device
    def partial(self, acc_in: Optional[torch.Tensor], W=None) -> torch.Tensor:
        """This key's rows reduced in arrival order ONTO ``acc_in`` (None:
        from +0), divided by fl32(W) when W is given; releases the rows.  The
        per-rank step of a client-sharded chain (fedsim_amd.sharding): rank r
        continues rank r-1's running sum, so no row may have been drained
        into the accumulator before (it would have started from +0)."""
        if acc_in is not None:
            if self.acc is not None:
                raise RuntimeError(
                    "rows were already drained from +0 (ring full): a chained partial sum "
                    "needs every row pending; raise slab_bytes / max_rows")
            self.acc = acc_in.reshape(-1)
        self._flush(final_W=W)
        out = self.acc
        self.release()
        self.acc = None
        return out

    @_on_own_device
    def pop_step(self, step: ops.ServerStep) -> None:
        """pop(on_device=True) followed by step.apply(avg), fused into the last
        drain when rows are pending, the step's operands allow it and the
        fused pass is the faster one at this size (ops.fuse_step_pays)."""
        if self.borrowed:
            fusable = step.aligned() and step.device == self.dev
            rows = len(self.borrowed)
        else:
            fusable = self.n_pending > 0 and ops.can_fuse_step(self.slab, step)
            rows = self.n_pending
        if not fusable or not ops.fuse_step_pays(self.P, rows, borrowed=bool(self.borrowed)):
            step.apply(self.pop(on_device=True).reshape(-1))
            return
        self._flush(final_W=self.cur_w if self._weighted() else None, step=step)
        self.release()
        self.acc = None


def _kernel_weight(weight) -> bool:
    """A weight the fp32 kernel applies exactly as the reference's
    ``value * weight`` does (fl32(weight) * value in fp32): a real Python or
    numpy number, or a real 0-dim host tensor (None raises in add, as in the
    reference)."""
    if weight is None or isinstance(weight, (int, float, np.integer, np.floating)):
        return True
    if isinstance(weight, torch.Tensor):
        # a 0-dim weight does not promote the value's dtype: fp32 * fl32(w)
        return weight.dim() == 0 and weight.device.type == "cpu" and not weight.is_complex()
    return False


def _kernel_value(value, weight) -> bool:
    """Whether (value, weight) is the fp32 kernel path's: an fp32 N-d tensor
    that does not require grad, and a real scalar weight.  A value that
    requires grad keeps the reference's arithmetic: its ``value * weight``
    (aggregators.py:21) carries the autograd graph into the sum and the
    quotient, which a kernel row cannot."""
    return (isinstance(value, torch.Tensor) and value.dim() > 0
            and value.dtype == torch.float32 and not value.requires_grad
            and _kernel_weight(weight))


def reference_add(pair, value, weight):
    """The reference's ``add`` on one key's (sum, weight) pair
    (fedsim/utils/aggregators.py:17-40, its evaluation order included):
    returns the new pair; raises, leaving nothing changed, where it does."""
    new_v, new_w = (value, None) if weight is None else (value * weight, weight)
    sum_v, cur_w = pair
    if (sum_v is None) or (new_v is None):
        return (sum_v + new_v, None)
    return (sum_v + new_v, cur_w + new_w)


# sums whose ``v / w`` ATen computes in f32 (its opmath type) on the CPU
_F32_OPMATH = (torch.float32, torch.float16, torch.bfloat16)


def reference_quotient(v, w):
    """The reference's ``v / w`` of get / pop (aggregators.py:58-60,
    120-122) for a sum ``v`` and a nonzero weight ``w``.  On the host it IS
    the reference's expression.  For a HIP tensor and a real Python / numpy
    weight it reproduces ATen CPU's rounding, which torch's HIP kernel (a
    multiply by the reciprocal) does not: the quotient's dtype is torch's
    promotion (an integer sum divides into the default float dtype), the
    division is IEEE true division in ATen's opmath type (f64 for fp64, f32
    for fp32 / fp16 / bf16) by the weight rounded to that type, then rounded
    to the quotient's dtype.  A sum that requires grad gets the reference's
    autograd node (``v / w``) holding these bits.  0-dim HIP sums (a
    metric kept on the GPU) divide the same way (round 6: found by the
    random sessions of tests/test_mixed_device.py)."""
    if not (isinstance(v, torch.Tensor) and v.device.type == "cuda" and not v.is_complex()):
        return v / w  # host values: the reference's own expression
    if isinstance(w, torch.Tensor):
        if (w.dim() != 0 or w.device.type != "cpu" or w.is_complex()
                or w.requires_grad):
            return v / w
    elif not isinstance(w, (int, float, np.integer, np.floating)):
        return v / w
    out = torch.result_type(v, w)
    if not out.is_floating_point:
        out = torch.get_default_dtype()  # true division of integers
    if isinstance(w, torch.Tensor):
        if out in (torch.float16, torch.bfloat16):
            # ATen CPU's reduced-float divide by a CPU scalar reads the
            # scalar's ORIGINAL value into opmath f32 (div_true_kernel,
            # original_scalar_value<opmath_t>): finalize applies fl32 to it
            w = w.item()
        else:
            # otherwise the 0-dim weight is first cast to the common dtype,
            # as ATen's TensorIterator does
            w = w.to(out).item()
    x = v.detach()
    if out == torch.float64:
        x = x.to(torch.float64).contiguous()
        q = ops.finalize_f64(x if x.data_ptr() % 16 == 0 else x.clone(), w)
    elif out in _F32_OPMATH:
        x = x.to(torch.float32).contiguous()
        q = ops.finalize(x if x.data_ptr() % 16 == 0 else x.clone(), w,
                         out=torch.empty(x.shape, dtype=torch.float32, device=x.device))
    else:
        return v / w
    q = q.view(v.shape).to(out)
    if v.requires_grad:
        g = v / w  # the reference's graph node (DivBackward saves v and w, not g)
        with torch.no_grad():
            g.copy_(q)
        return g
    return q


def _ref_weight(weight) -> bool:
    """A weight fedagg_reduce_rows_ref applies as ATen does: a real Python or
    numpy number (converted to the opmath type)."""
    return isinstance(weight, (int, float, np.integer, np.floating)) and not isinstance(
        weight, complex)


class _RefDeviceEntry(_TensorEntry):
    """A HIP-resident key of bf16 / fp16 / fp64 tensors with real scalar
    weights: the reference's arithmetic (aggregators.py:17-40, every product
    and every sum rounded to the dtype, in arrival order) by
    fedagg_reduce_rows_ref, in HBM, instead of two torch launches and three
    passes per client.  ``add`` snapshots the value (the reference's clone,
    training/utils.py:34) unless the aggregator borrows handed-over HBM
    tensors; rows are reduced onto the running sum when ``max_rows`` or the
    HBM budget are reached and at get / pop.  The sum and the quotient
    (reference_quotient) are bitwise the reference's CPU tensors."""

    DTYPES = (torch.bfloat16, torch.float16, torch.float64)

    def __init__(self, value: torch.Tensor, opts: _Options):
        self.shape = tuple(value.shape)
        self.dtype = value.dtype
        self.dev = value.device
        self.out_device = value.device
        self.P = value.numel()
        self.borrow = opts.borrow
        budget = _slab_budget(self.dev, opts.slab_bytes)
        self.Bmax = max(1, min(opts.max_rows, budget // max(1, self.P * value.element_size())))
        self.rows: List = []  # (tensor, version or None)
        self.ws: List = []
        self.acc: Optional[torch.Tensor] = None
        self.cur_w = 0

    def takes(self, value, weight) -> bool:
        return (isinstance(value, torch.Tensor) and value.dtype == self.dtype
                and value.device == self.dev and tuple(value.shape) == self.shape
                and not value.requires_grad and _ref_weight(weight))

    @_on_own_device
    def add(self, value: torch.Tensor, weight) -> None:
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        src = value.detach() if value.requires_grad else value
        # rows are read flat by data pointer: no reshape view (~1 us per add)
        if self.borrow and src.is_contiguous():
            row = (src, src._version)  # handed over: read at the reduction
        else:
            row = (src.clone(memory_format=torch.contiguous_format), None)
        self.rows.append(row)
        self.ws.append(weight)
        self.cur_w = new_w
        if len(self.rows) >= self.Bmax:
            self._drain()

    def _drain(self) -> None:
        if not self.rows:
            return
        rows = []
        for t, version in self.rows:
            if version is not None and t._version != version:
                raise RuntimeError(
                    "a client tensor was modified in place after SerialAggregator.add(); "
                    "an aggregator created with borrow=True reads it when the round is "
                    "reduced (use borrow=False to snapshot it at add time)")
            rows.append(t)
        out = self.acc if self.acc is not None else torch.empty(self.P, dtype=self.dtype,
                                                                device=self.dev)
        ops.reduce_rows_ref(rows, self.ws, out, acc_in=self.acc)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        _keep_until(ev, rows)  # the rows stay alive until the reduction ran
        self.acc = out
        self.rows, self.ws = [], []

    def _weighted(self) -> bool:
        return not (self.cur_w is None or self.cur_w == 0)

    @_on_own_device
    def get_sum(self) -> torch.Tensor:
        self._drain()
        return self.acc.view(self.shape).clone()

    @_on_own_device
    def get(self) -> torch.Tensor:
        s = self.get_sum()
        return reference_quotient(s, self.cur_w) if self._weighted() else s

    @_on_own_device
    def pop(self, on_device: bool = False) -> torch.Tensor:
        self._drain()
        s = self.acc.view(self.shape)
        self.acc = None
        return reference_quotient(s, self.cur_w) if self._weighted() else s

    @_on_own_device
    def pop_step(self, step: ops.ServerStep) -> None:
        step.apply(self.pop().reshape(-1).to(step.device, torch.float32).contiguous())


def _drop_entry(entry) -> None:
    release = getattr(entry, "release", None)
    if release is not None:
        release()


class SerialAggregator(object):
    """Device-backed drop-in for the reference SerialAggregator
    (fedsim/utils/aggregators.py:11-144).

    Args:
        device: HIP device for tensor keys (default: the tensor's own device if
            it is a HIP tensor, else the current HIP device).
        slab_bytes: HBM budget of the pending-row ring per key; when it fills,
            pending rows are reduced into the accumulator (order is preserved).
        max_rows: cap on ring rows per key.
        flags: libfedagg tuning flags (include/fedagg.h); default = tuned per C.
        expected_rows: hint (e.g. clients per round) to size the ring once.
        block_cols: column-block width C of the slab (1024 / 2048 / 4096);
            default = ops.choose_block_cols(P).
        borrow: reduce HBM-resident client tensors where they are instead of
            snapshotting them into the slab at ``add`` (no copy: the round
            reads 4 B per client element instead of 12).  The caller hands the
            tensor over: modifying it in place after ``add`` makes the next
            reduction raise (torch's version counter is checked).  The round
            driver enables it, since its client messages are dropped right
            after ``receive_from_client``.
        borrow_host: the same hand-over for host tensors: ``add`` returns
            before the vector is copied into pinned staging; the ingest
            worker copies and DMAs it while the caller goes on (the next
            client trains).  Modifying it in place before that copy raises at
            the reduction.  The round driver enables it; serial_aggregation
            clones a vector whose ownership it cannot show.
        fast: for models too small for one column per lane to fill the chip
            (P below 65,536), split each column's K clients over several waves
            (FEDAGG_FAST).  Deterministic, but the summation order is no longer
            the reference's: results match it normwise (<= 1e-6 relative), not
            bit for bit.  No effect at larger P.
    """

    def __init__(self, device=None, slab_bytes: Optional[int] = _DEFAULT_SLAB_BYTES,
                 max_rows: int = _DEFAULT_MAX_ROWS, flags: Optional[int] = None,
                 expected_rows: Optional[int] = None,
                 block_cols: Optional[int] = None, borrow: bool = False,
                 fast: bool = False, borrow_host: bool = False) -> None:
        self._members: Dict = dict()
        self._reserved: Dict = dict()  # keys with reserved rows but no add yet
        self._opts = _Options(device, slab_bytes, max_rows, flags, expected_rows, block_cols,
                              borrow, fast, borrow_host)
    @staticmethod
    def _ingest(dev) -> _Ingest:
        return _ingest_for(dev)

    def _new_entry(self, value: torch.Tensor) -> _TensorEntry:
        """State of a new tensor-valued key (sharded aggregators override)."""
        return _DeviceEntry(value, _hip_device(value, self._opts.device), self._opts, self)

    def _new_ref_entry(self, value, weight) -> Optional[_TensorEntry]:
        """A HIP bf16 / fp16 / fp64 key with a real scalar weight: the
        reference's arithmetic in HBM (_RefDeviceEntry); None otherwise (the
        sharded aggregators keep such keys on the host path)."""
        if (isinstance(value, torch.Tensor) and value.dim() > 0 and value.device.type == "cuda"
                and value.dtype in _RefDeviceEntry.DTYPES and _ref_weight(weight)
                and type(value) is torch.Tensor and not value.requires_grad):
            return _RefDeviceEntry(value, self._opts)
        return None

    @staticmethod
    def _is_device_value(value, weight=1) -> bool:
        """Whether an add of (value, weight) to a new key starts a kernel
        entry (an fp32 N-d tensor with a real scalar weight)."""
        return _kernel_value(value, weight)

    def reserve(self, key, P: int, device) -> Optional[SlabRow]:
        """A row of ``key``'s HBM ring for a client to write its P-parameter
        vector into (slab_rows.reserve_round_row / vectorize_module(out=)),
        or None if this key cannot take one (not part of the reference API).
        The key does not exist for ``in`` / ``pop_all`` until a value is
        added."""
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        e = self._members.get(key)
        if e is None:
            e = self._reserved.get(key)
            if e is not None and (e.P != P or e.dev != dev):
                # a reservation for another size / device that was never
                # added: drop it (live rows keep a copy) and start over
                e.release()
                del self._reserved[key]
                e = None
        if e is None:
            like = _Like((P,), dev)
            e = _DeviceEntry(like, _hip_device(like, self._opts.device), self._opts, self)
            if e.dev != dev:
                return None
            self._reserved[key] = e
        if type(e) is not _DeviceEntry or e.P != P or e.dev != dev or e.shape != (P,):
            return None
        return e.reserve()

    def add(self, key, value, weight=None):
        entry = self._members.get(key)
        if entry is None and key in self._reserved:
            res = self._reserved.pop(key)
            if self._is_device_value(value, weight) and tuple(value.shape) == res.shape:
                # the first add defines the key, as in the reference: adopt
                # the reserved ring only for a value of its shape
                entry = self._members[key] = res
                entry.out_device = value.device  # results go where the first value came from
            else:
                res.release()  # a reserved row still alive keeps a copy
        if isinstance(entry, _TensorEntry):
            if entry.takes(value, weight):
                entry.add(value, weight)
                return
            # the key leaves the kernel path (a value of another dtype or
            # shape, a scalar, a non-real weight): its exact running sum so
            # far continues under the reference's arithmetic, which applies
            # torch's promotion / broadcasting -- or raises -- as there
            pair = reference_add((entry.get_sum(), entry.cur_w), value, weight)
            _drop_entry(entry)
            self._members[key] = pair
            return
        if entry is None and self._is_device_value(value, weight):
            entry = self._new_entry(value)
            entry.add(value, weight)
            self._members[key] = entry
            return
        if entry is None:
            entry = self._new_ref_entry(value, weight)
            if entry is not None:
                entry.add(value, weight)  # may raise (weight None): the key is not created
                self._members[key] = entry
                return
        # the reference's own arithmetic (aggregators.py:17-40) on the
        # value's device: scalars, 0-dim tensors, host tensors of other dtypes
        self._members[key] = reference_add(self._members.get(key, (0, 0)), value, weight)

    def _entry(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        return self._members[key]

    def get(self, key):
        e = self._entry(key)
        if isinstance(e, _TensorEntry):
            return e.get()
        v, w = e
        if w is None or w == 0:
            return v
        return reference_quotient(v, w)

    def get_sum(self, key):
        e = self._entry(key)
        if isinstance(e, _TensorEntry):
            return e.get_sum()
        return e[0]

    def get_weight(self, key):
        e = self._entry(key)
        if isinstance(e, _TensorEntry):
            return e.cur_w
        return e[1]

    def keys(self):
        return self._members.keys()

    def pop(self, key):
        e = self._entry(key)
        del self._members[key]
        if isinstance(e, _TensorEntry):
            return e.pop()
        v, w = e
        if w is None or w == 0:
            return v
        return reference_quotient(v, w)

    def pop_device(self, key):
        """``pop`` that leaves a tensor result in HBM (no D2H), for the fused
        server step (not part of the reference API)."""
        e = self._entry(key)
        if not isinstance(e, _TensorEntry):
            return self.pop(key)
        del self._members[key]
        return e.pop(on_device=True)

    def device_of(self, key) -> Optional[torch.device]:
        """HIP device holding a tensor key's sum (None for host keys)."""
        e = self._entry(key)
        return e.dev if isinstance(e, _TensorEntry) else None

    def pop_step(self, key, step: ops.ServerStep) -> None:
        """``pop(key)`` and ``step.apply(average)`` in one pass over the
        pending client rows (not part of the reference API): the server step
        of FedAvg / AdaBest / FedNova / FedDyn optimize runs in the epilogue of
        the round's last reduction, so the average is never stored."""
        e = self._entry(key)
        if not isinstance(e, _TensorEntry):
            avg = self.pop(key)
            step.apply(avg.reshape(-1).to(step.device, torch.float32).contiguous())
            return
        del self._members[key]
        if e.dev != step.device:
            step.apply(e.pop(on_device=True).reshape(-1).to(step.device))
            return
        e.pop_step(step)

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
        # the reference slices [-min(k, n):], so k=0 (a -0 slice) means "all"
        n = len(list_v) if k is None else min(k, len(list_v))
        vs, ws = list_v[-n:], list_w[-n:]
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
