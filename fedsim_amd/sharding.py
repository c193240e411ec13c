"""Multi-GPU decompositions of the aggregation.

One process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL on
ROCm, over xGMI).  Three modes:

* ``param``   parameter-sharded.  Rank g owns the contiguous column range
              ``shard_range(P, g, N)`` of every client row and reduces all K
              clients over it.  No collective on the data path; per-column
              order is unchanged, so the result is BIT-EXACT.  (Config 4.)
* ``chain``   client-sharded, bit-exact.  Rank g holds clients
              ``shard_range(K, g, N)``.  The accumulator is pipelined through
              the ranks in column blocks: rank g receives block j's running sum
              from rank g-1, adds its own clients (in arrival order) and sends
              it on; the last rank finalizes.  Every column still sees
              k = 0..K-1 in order.  Traffic per block is 4*P/M bytes over one
              point-to-point xGMI hop, hidden behind the block's reduction.
* ``allreduce`` client-sharded, reordered.  Each rank reduces its clients into
              a partial fp32 sum, then one RCCL all-reduce(sum) of 4P bytes and
              the divide by fl32(W).  Summation order changes, so parity is
              normwise (||y - y_ref|| / ||y_ref|| <= 1e-6).  (Config 5.)

The per-rank reduction is the HIP kernel: ``ops.reduce_blocked`` on a
column-blocked slab ([nblk, Kcap, C], the layout the aggregator packs into and
the bench times), ``ops.reduce_slab`` on a row-major [K, P] view;
``param_sharded_step`` runs the round's server step fused into the shard's
pass (fedagg_reduce_step_blocked_f32).  ``local_reduce`` can be injected so the
host-side protocol is testable with gloo on CPU.

On the plugin surface, ``ShardedSerialAggregator`` is the SerialAggregator
drop-in whose tensor keys are parameter-sharded over the ranks of a process
group (see its docstring).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

from . import ops

ALIGN = 64  # fp32 columns: shard boundaries on 256-B lines


def shard_range(n: int, rank: int, world: int, align: int = 1):
    """Contiguous [lo, hi) of ``n`` items for ``rank``; interior boundaries are
    multiples of ``align`` (the last shard takes the remainder)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    units = (n + align - 1) // align
    lo_u = units * rank // world
    hi_u = units * (rank + 1) // world
    lo, hi = min(n, lo_u * align), min(n, hi_u * align)
    return lo, hi


def shard_span(n: int, rank: int, world: int, align: int = ALIGN):
    """[lo, hi) of ``n`` columns for ``rank`` when every shard but the last has
    the same width S = ceil(ceil(n / align) / world) * align: equal widths let
    the ranks exchange their shards with one all-gather of world * S columns.
    A rank past the end gets an empty span (lo == hi == n)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    S = shard_width(n, world, align)
    return min(n, rank * S), min(n, (rank + 1) * S)


def shard_width(n: int, world: int, align: int = ALIGN) -> int:
    units = (n + align - 1) // align
    return (units + world - 1) // world * align


def _hip_reduce(X, w32, out, acc_in=None, W=None, flags=0):
    """The per-rank HIP reduction: column-blocked slab ([nblk, Kcap, C], the
    tuned layout) or a row-major [K, P] view."""
    if X.dim() == 3:
        return ops.reduce_blocked(X, w32, out, B=min(X.shape[1], w32.numel()), acc_in=acc_in,
                                  W=W, flags=flags or ops.default_flags(X.shape[2]))
    return ops.reduce_slab(X, w32, out, acc_in=acc_in, W=W, P=out.numel(), flags=flags)


def param_sharded(X_shard: torch.Tensor, w32: torch.Tensor, W, out_shard: torch.Tensor,
                  local_reduce: Callable = _hip_reduce, flags: int = 0) -> torch.Tensor:
    """Reduce this rank's column shard of all K clients (no collective)."""
    return local_reduce(X_shard, w32, out_shard, None, W, flags)


def param_sharded_step(Xb_shard: torch.Tensor, w32: torch.Tensor, W, step: "ops.ServerStep",
                       B: Optional[int] = None, acc_in: Optional[torch.Tensor] = None,
                       avg: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One rank's share of a parameter-sharded round: reduce this rank's
    column shard (column-blocked slab [nblk, Kcap, C]) of B clients, divide by
    fl32(W) and run the server step on the shard's slice of the cloud
    (``step`` = the full step narrowed to the shard, ServerStep.narrow).  One
    pass (fedagg_reduce_step_blocked_f32) where ops.fuse_step_pays, else the
    stored average (``avg``, allocated if None) and fedagg_server_step_f32;
    same bits either way.  No collective; bitwise equal to the reference."""
    B = Xb_shard.shape[1] if B is None else B
    if ops.fuse_step_pays(step.P, B) and ops.can_fuse_step(Xb_shard, step):
        return ops.reduce_blocked_step(Xb_shard, w32, step, B=B, acc_in=acc_in, W=W)
    if avg is None:
        avg = torch.empty(step.P, dtype=torch.float32, device=Xb_shard.device)
    ops.reduce_blocked(Xb_shard, w32, avg, B=B, acc_in=acc_in, W=W,
                       flags=ops.default_flags(Xb_shard.shape[2]))
    return step.apply(avg)


def client_sharded_allreduce(X_local: torch.Tensor, w32_local: torch.Tensor, W,
                             out: torch.Tensor, group=None,
                             local_reduce: Callable = _hip_reduce,
                             flags: int = 0) -> torch.Tensor:
    """Partial sum of this rank's clients -> all-reduce(sum) -> divide by fl32(W)."""
    local_reduce(X_local, w32_local, out, None, None, flags)
    dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
    if W is not None and W != 0:
        if out.device.type == "cuda":
            ops.finalize(out, W, out=out)
        else:  # CPU gloo rehearsal of the protocol
            out.div_(ops.fl32(W))
    return out


def client_sharded_chain(X_local: torch.Tensor, w32_local: torch.Tensor, W,
                         out: torch.Tensor, n_blocks: int = 64, group=None,
                         local_reduce: Callable = _hip_reduce,
                         flags: int = 0) -> Optional[torch.Tensor]:
    """Bit-exact client-sharded reduction, pipelined through the ranks.

    Rank r reduces its own clients into each column block after receiving the
    running sum of ranks 0..r-1 for that block.  The final (finalized) result
    is produced on the last rank and broadcast to all ranks in ``out``.
    """
    if X_local.dim() != 2:
        raise ValueError("client_sharded_chain takes row-major [K_local, P] client rows "
                         "(its column blocks are column slices of them)")
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    P = out.numel()
    last = world - 1
    reqs = []
    for j in range(n_blocks):
        lo, hi = shard_range(P, j, n_blocks, ALIGN)
        if hi <= lo:
            continue
        blk = out[lo:hi]
        if rank > 0:
            dist.recv(blk, src=rank - 1, group=group)
        acc_in = None if rank == 0 else blk
        local_reduce(X_local[:, lo:hi], w32_local, blk, acc_in,
                     W if rank == last else None, flags)
        if rank < last:
            reqs.append(dist.isend(blk, dst=rank + 1, group=group))
    for r in reqs:
        r.wait()
    dist.broadcast(out, src=last, group=group)
    return out


def weights_fp32(weights: Sequence, device) -> torch.Tensor:
    return torch.tensor([ops.fl32(w) for w in weights], dtype=torch.float32, device=device)


# ---------------------------------------------------------------------------
# plugin surface: a parameter-sharded SerialAggregator
# ---------------------------------------------------------------------------
from .utils.aggregators import (  # noqa: E402
    SerialAggregator, _deliver_to, _DeviceEntry, _hip_device, _kernel_value, _ref_weight,
    _RefDeviceEntry, _TensorEntry, reference_add, reference_quotient)


def _group_rank_world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    if group is not None:
        raise RuntimeError("a process group was given but torch.distributed is not initialised")
    return 0, 1


class _ShardEntry(_TensorEntry):
    """One tensor-valued key of a ShardedSerialAggregator: this rank reduces
    columns [lo, hi) of every client vector (``inner``, a one-GPU entry on its
    own device); results are assembled with one all-gather of the equal-width
    shards."""

    def __init__(self, agg: "ShardedSerialAggregator", value: torch.Tensor, ref: bool = False):
        self.agg = agg
        self.shape = tuple(value.shape)
        self.P = value.numel()
        self.dtype = value.dtype if ref else torch.float32
        self.ref = ref  # a bf16 / fp16 / fp64 key: _RefDeviceEntry on the slice
        self.out_device = value.device
        self.lo, self.hi = shard_span(self.P, agg._rank, agg._world)
        self.S = shard_width(self.P, agg._world)
        self.cur_w = 0
        part = value.reshape(-1)[self.lo:self.hi]
        self.inner = None if self.hi <= self.lo else (
            _RefDeviceEntry(part, agg._opts) if ref else agg._shard_entry(part))
        self.dev = self.inner.dev if self.inner is not None else agg._device_for(value)

    def takes(self, value, weight) -> bool:
        if not self.ref:
            return super().takes(value, weight)
        return (isinstance(value, torch.Tensor) and value.dtype == self.dtype
                and value.device == self.out_device and tuple(value.shape) == self.shape
                and not value.requires_grad and _ref_weight(weight))

    def add(self, value: torch.Tensor, weight) -> None:
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        if tuple(value.shape) != self.shape:
            raise ValueError(
                f"tensor of shape {tuple(value.shape)} added to a key aggregating {self.shape}")
        if self.inner is not None:
            src = value.detach() if value.requires_grad else value
            self.inner.add(src.reshape(-1)[self.lo:self.hi], weight)
        self.cur_w = new_w

    # -- exchange -----------------------------------------------------------
    def _gather_into(self, full: torch.Tensor, part: Optional[torch.Tensor]) -> torch.Tensor:
        """full[lo:hi] = part on this rank, then every rank's shard into
        ``full`` (one all-gather of world x S columns)."""
        if part is not None and part.data_ptr() != full[self.lo:self.hi].data_ptr():
            full[self.lo:self.hi].copy_(part.reshape(-1))
        if self.agg._world == 1:
            return full
        # gloo has no all-gather of HIP tensors: such groups exchange the
        # shards through host memory (RCCL groups gather in HBM over xGMI)
        via_host = full.device.type == "cuda" and \
            dist.get_backend(self.agg._group) == dist.Backend.GLOO
        mine = torch.zeros(self.S, dtype=full.dtype, device="cpu" if via_host else full.device)
        mine[: self.hi - self.lo].copy_(full[self.lo:self.hi])
        ws = mine.new_empty(self.agg._world * self.S)
        dist.all_gather_into_tensor(ws, mine, group=self.agg._group)
        full.copy_(ws[: self.P])
        return full

    def _assemble(self, part: Optional[torch.Tensor]) -> torch.Tensor:
        full = torch.empty(self.P, dtype=self.dtype, device=self.dev)
        self._gather_into(full, part)
        return full

    def _deliver(self, t: torch.Tensor) -> torch.Tensor:
        return _deliver_to(t.view(self.shape), self.out_device)

    # -- reference semantics --------------------------------------------------
    def get(self) -> torch.Tensor:
        return self._deliver(self._assemble(None if self.inner is None else self.inner.get()))

    def get_sum(self) -> torch.Tensor:
        part = None if self.inner is None else self.inner.get_sum()
        return self._deliver(self._assemble(part))

    def pop(self, on_device: bool = False) -> torch.Tensor:
        part = None if self.inner is None else self.inner.pop(on_device=True)
        full = self._assemble(part)
        return full.view(self.shape) if on_device else self._deliver(full)

    def pop_step(self, step: ops.ServerStep) -> None:
        """This rank's shard of pop + server step (ServerStep.narrow), then
        every operand the step wrote is re-assembled on every rank, all of
        them in ONE all-gather (a [n_operands, S] block per rank)."""
        if self.inner is not None:
            self.inner.pop_step(step.narrow(self.lo, self.hi))
        outs = step.outputs()
        if self.agg._world == 1:
            return
        if len(outs) == 1:
            self._gather_into(outs[0], None)
            return
        full0 = outs[0]
        via_host = full0.device.type == "cuda" and \
            dist.get_backend(self.agg._group) == dist.Backend.GLOO
        n, S, width = len(outs), self.S, self.hi - self.lo
        mine = torch.zeros((n, S), dtype=full0.dtype, device="cpu" if via_host else full0.device)
        for j, t in enumerate(outs):
            mine[j, :width].copy_(t[self.lo:self.hi])
        ws = mine.new_empty((self.agg._world, n, S))
        dist.all_gather_into_tensor(ws.view(-1), mine.view(-1), group=self.agg._group)
        for j, t in enumerate(outs):
            # rank r's shard of operand j is ws[r, j, :]: the ranks' shards
            # are consecutive S-column spans of [0, P)
            t.copy_(ws[:, j, :].reshape(-1)[: self.P])


class _DevicesEntry(_TensorEntry):
    """One tensor key of a single-process ShardedSerialAggregator over
    several local GPUs: shard i (columns [lo_i, hi_i)) is reduced by a
    one-GPU entry on devices[i]; results are assembled by copies between the
    devices (or into one pinned host tensor)."""

    def __init__(self, agg: "ShardedSerialAggregator", value: torch.Tensor):
        self.agg = agg
        self.shape = tuple(value.shape)
        self.P = value.numel()
        self.out_device = value.device
        n = len(agg._devices)
        self.spans = [shard_span(self.P, i, n) for i in range(n)]
        flat = value.reshape(-1)
        self.inners = [None if hi <= lo else
                       _DeviceEntry(flat[lo:hi], dev, agg._opts, agg, out_device=dev)
                       for (lo, hi), dev in zip(self.spans, agg._devices)]
        self.cur_w = 0

    @property
    def dev(self):
        """Where the server step's operands should live: with the results
        (the host for a host-resident run: each GPU then moves only its
        slice over its own link)."""
        return self.out_device

    def add(self, value: torch.Tensor, weight) -> None:
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        if tuple(value.shape) != self.shape:
            raise ValueError(
                f"tensor of shape {tuple(value.shape)} added to a key aggregating {self.shape}")
        src = value.detach() if value.requires_grad else value
        flat = src.reshape(-1)
        for (lo, hi), inner in zip(self.spans, self.inners):
            if inner is not None:
                with torch.cuda.device(inner.dev):  # its launches: its device current
                    inner.add(flat[lo:hi], weight)  # host slices: each GPU's own copy stream
        self.cur_w = new_w

    def _each(self, fn):
        """fn(inner) for every shard, with that shard's GPU as the current
        device: libfedagg launches on the stream it is handed, and HIP
        launches go to the current device's queues."""
        out = []
        for inner in self.inners:
            if inner is None:
                out.append(None)
                continue
            with torch.cuda.device(inner.dev):
                out.append(fn(inner))
        return out

    def _assemble(self, parts, on=None) -> torch.Tensor:
        on = self.out_device if on is None else on
        host = on.type == "cpu"
        full = torch.empty(self.P, dtype=torch.float32, device=on, pin_memory=host)
        for (lo, hi), part in zip(self.spans, parts):
            if part is not None:
                full[lo:hi].copy_(part.reshape(-1), non_blocking=host)
        if host:
            for inner in self.inners:
                if inner is not None:
                    torch.cuda.current_stream(inner.dev).synchronize()
        return full

    def get(self) -> torch.Tensor:
        return self._assemble(self._each(lambda e: e.get())).view(self.shape)

    def get_sum(self) -> torch.Tensor:
        return self._assemble(self._each(lambda e: e.get_sum())).view(self.shape)

    def pop(self, on_device: bool = False) -> torch.Tensor:
        parts = self._each(lambda e: e.pop(on_device=True))
        return self._assemble(parts).view(self.shape)

    def pop_step(self, step: ops.ServerStep) -> None:
        """Each GPU runs the step on its slice: in place when the operands
        live on that GPU, else on a copy of the operand slices moved over
        that GPU's own link (PCIe for a host-resident cloud), copied back."""
        home = step.device
        back = []
        for (lo, hi), inner in zip(self.spans, self.inners):
            if inner is None:
                continue
            sub = step.narrow(lo, hi)
            with torch.cuda.device(inner.dev):
                if inner.dev != home:
                    moved = {n: t.to(inner.dev, non_blocking=True)
                             for n, t in sub.operands.items()}
                    local = ops.ServerStep(step.algo, moved.pop("cloud"), **step._scalars,
                                           **moved)
                    inner.pop_step(local)
                    back.append((sub, local, inner.dev))
                else:
                    inner.pop_step(sub)
        for sub, local, dev in back:
            host = home.type == "cpu"
            with torch.cuda.device(dev):
                for name, t in local.operands.items():
                    sub.operands[name].copy_(t, non_blocking=host)
                if host:
                    torch.cuda.current_stream(dev).synchronize()


class ShardedSerialAggregator(SerialAggregator):
    """Parameter-sharded drop-in for the reference SerialAggregator
    (fedsim/utils/aggregators.py:11-144) over the ranks of a process group,
    one process per GPU (the reference round loop it serves is
    fedsim/distributed/centralized/centralized_fl_algorithm.py:411-443).

    Every rank runs the same round (SPMD) and is handed every client vector;
    rank g keeps only columns [lo_g, hi_g) of each (``shard_span``: 64-column
    aligned, equal widths but the last):

    * a host vector crosses PCIe as that slice only, on this GPU's own copy
      stream and link, so N ranks ingest over N links at once;
    * a vector already in this GPU's HBM is reduced in place (``borrow``) or
      packed from there; the slice of a 256-B aligned vector stays aligned;
    * the reduction is the one-GPU path on the slice (column-blocked ring
      slab or borrowed rows, exact mode), so every column keeps the reference's
      summation order: results are BIT-EXACT, with no collective on the data
      path;
    * ``pop_step`` runs the round's server step on the slice (fused into the
      last pass where that pays) and then assembles every operand it wrote
      (cloud, its pseudo-gradient, aux / momentum state) with one all-gather
      each, so every rank holds the full new model for the next round;
    * ``get`` / ``get_sum`` / ``pop`` assemble the average the same way and
      deliver it on the device the values came from.

    Scalar keys (the per-split metrics) stay on the host with the
    reference's arithmetic, identically on every rank.

    Single-process mode (``devices=[...]``): one process drives several
    local GPUs, shard i on devices[i] -- for FedSim's own single-process
    simulator.  Host client vectors cross PCIe slice by slice, one link per
    GPU; the server step runs on each GPU's slice of the cloud (moved over
    that GPU's link when the cloud lives on the host) and the results are
    assembled in one pinned host tensor (or on the cloud's GPU).  HBM
    vectors of one GPU reach the other shards over xGMI.

    Args:
        group: the torch.distributed group (default: the default group; a
            single process with no group is world 1).
        devices: single-process mode (see above); excludes ``group``.
        entry_factory: TEST HOOK.  ``entry_factory(slice, agg)`` builds the
            per-rank state of a key instead of the HIP entry, so the protocol
            can be rehearsed with gloo on CPU (tests/test_sharding_gloo.py).
        **kwargs: SerialAggregator's options, applied to each rank's slice.
    """

    def __init__(self, group=None, entry_factory: Optional[Callable] = None,
                 devices: Optional[Sequence] = None, **kwargs) -> None:
        super().__init__(**kwargs)
        self._devices = None
        if devices is not None:
            if group is not None or entry_factory is not None:
                raise ValueError("devices= is the single-process mode: no group / entry_factory")
            self._devices = [torch.device(d) for d in devices]
            if not self._devices or any(d.type != "cuda" for d in self._devices):
                raise ValueError("devices must be one or more HIP devices")
            self._group, self._rank, self._world = None, 0, 1
        else:
            self._group = group
            self._rank, self._world = _group_rank_world(group)
        self._entry_factory = entry_factory

    def _device_for(self, value: torch.Tensor) -> torch.device:
        if self._entry_factory is not None:
            return value.device
        return _hip_device(value, self._opts.device)

    def _shard_entry(self, part: torch.Tensor) -> _TensorEntry:
        if self._entry_factory is not None:
            return self._entry_factory(part, self)
        dev = _hip_device(part, self._opts.device)
        return _DeviceEntry(part, dev, self._opts, self, out_device=dev)

    def _new_entry(self, value: torch.Tensor) -> _TensorEntry:
        if self._devices is not None:
            return _DevicesEntry(self, value)
        return _ShardEntry(self, value)

    def reserve(self, key, P, device):
        """Client rows are not reserved in a sharded round (each rank keeps a
        column slice of every vector, not whole rows)."""
        return None

    def _new_ref_entry(self, value, weight):
        """A HIP bf16 / fp16 / fp64 key with a real scalar weight: each rank
        reduces its column slice with the reference's arithmetic
        (_RefDeviceEntry), assembled like the fp32 keys.  Single-process
        shards keep such keys on the host path."""
        if self._devices is not None or self._entry_factory is not None:
            return None
        if (isinstance(value, torch.Tensor) and value.dim() > 0 and value.device.type == "cuda"
                and value.dtype in _RefDeviceEntry.DTYPES and _ref_weight(weight)
                and type(value) is torch.Tensor and not value.requires_grad):
            return _ShardEntry(self, value, ref=True)
        return None

    @property
    def rank(self) -> int:
        return self._rank

    @property
    def world_size(self) -> int:
        return self._world

    def shard_of(self, key):
        """[lo, hi) columns this rank reduces for a tensor key."""
        e = self._entry(key)
        return (e.lo, e.hi) if isinstance(e, _ShardEntry) else None


# ---------------------------------------------------------------------------
# client-sharded rounds on the plugin surface
# ---------------------------------------------------------------------------
class RemoteRow(torch.Tensor):
    """Stand-in for a client vector that lives on another rank of a
    client-sharded round: shape and dtype only, no storage (a wrapper over
    the meta device).  Copies and detaches keep the stand-in (the reference's
    ``clone().detach().data``, training/utils.py:34, feddf.py:87); any
    arithmetic on it raises, naming the rank that holds the vector."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    @staticmethod
    def __new__(cls, shape, dtype, src_type: str, owner: int):
        t = torch.Tensor._make_wrapper_subclass(cls, tuple(shape), dtype=dtype, device="meta")
        t.src_type = src_type  # "cuda" / "cpu": where the client produced it
        t.owner = owner
        return t

    def __repr__(self):
        return "RemoteRow(shape=%s, owner=rank %d)" % (tuple(self.shape), self.owner)

    @classmethod
    def __torch_dispatch__(cls, func, types, args=(), kwargs=None):
        src = args[0]
        if func in _REMOTE_KEEP:
            return RemoteRow(src.shape, src.dtype, src.src_type, src.owner)
        raise RuntimeError(
            f"{func} on a client vector held by rank {src.owner} of a client-sharded round: "
            "only its SerialAggregator can use it")


_aten = torch.ops.aten
_REMOTE_KEEP = (_aten.clone.default, _aten.detach.default, _aten.alias.default)


class _RowStub(object):
    """Picklable description of a message tensor (RemoteRow on arrival)."""

    __slots__ = ("shape", "dtype", "src_type", "owner")

    def __init__(self, t: torch.Tensor, owner: int):
        self.shape, self.dtype, self.src_type, self.owner = (
            tuple(t.shape), t.dtype, t.device.type, owner)


class _ScalarTensor(object):
    """A 0-dim message tensor (a metric) sent by value."""

    __slots__ = ("value", "src_type")

    def __init__(self, t: torch.Tensor):
        self.value, self.src_type = t.detach().cpu(), t.device.type


def _skeleton(obj, owner: int):
    if isinstance(obj, torch.Tensor):
        return _ScalarTensor(obj) if obj.dim() == 0 else _RowStub(obj, owner)
    if isinstance(obj, dict):
        return {k: _skeleton(v, owner) for k, v in obj.items()}
    if type(obj) in (list, tuple):
        return type(obj)(_skeleton(v, owner) for v in obj)
    return obj


def _flesh(obj, device):
    if isinstance(obj, _RowStub):
        return RemoteRow(obj.shape, obj.dtype, obj.src_type, obj.owner)
    if isinstance(obj, _ScalarTensor):
        return obj.value.to(device) if obj.src_type == "cuda" and device.type == "cuda" \
            else obj.value
    if isinstance(obj, dict):
        return {k: _flesh(v, device) for k, v in obj.items()}
    if type(obj) in (list, tuple):
        return type(obj)(_flesh(v, device) for v in obj)
    return obj


def _global_rank(group, r: int) -> int:
    return r if group is None else dist.get_global_rank(group, r)


def _via_host(group, t: torch.Tensor) -> bool:
    """gloo moves host tensors only: HIP tensors of a gloo group go through
    host memory (RCCL groups move them in HBM over xGMI)."""
    return t.device.type == "cuda" and dist.get_backend(group) == dist.Backend.GLOO


def _send(t, dst, group):
    dist.send(t.cpu() if _via_host(group, t) else t, dst=dst, group=group)


def _recv(t, src, group):
    if _via_host(group, t):
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.recv(t, src=src, group=group)


def _broadcast(t, src, group):
    if _via_host(group, t):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=group)


def _all_reduce_sum(t, group):
    if _via_host(group, t):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


class _ClientShardEntry(_TensorEntry):
    """A tensor key of a client-sharded round: the Python weight sum over
    every client of the round in arrival order (the reference's ``cur_w``),
    which ranks hold rows in that order, and this rank's own rows as a
    one-GPU entry (exact, arrival order)."""

    def __init__(self, agg: "ClientShardedSerialAggregator", shape, src_type: str):
        self.agg = agg
        self.shape = tuple(shape)
        self.P = 1
        for d in self.shape:
            self.P *= d
        self.src_type = src_type
        self.dev = agg._reduce_device()
        self.out_device = self.dev if src_type == "cuda" else torch.device("cpu")
        self.cur_w = 0
        self.local = None
        self.owners = []  # ranks holding rows, in arrival order (one run each)
        self.sum = None

    def _owner(self, r: int) -> None:
        if not self.owners or self.owners[-1] != r:
            self.owners.append(r)

    def add(self, value: torch.Tensor, weight) -> None:
        new_w = self.cur_w + weight  # TypeError for weight=None, as the reference
        if tuple(value.shape) != self.shape:
            raise ValueError(
                f"tensor of shape {tuple(value.shape)} added to a key aggregating {self.shape}")
        if self.sum is not None:
            # the rows were combined across ranks by a get / get_sum: a later
            # row would have to be chained onto that sum on its owner, which
            # this round protocol does not do -- refuse rather than drop it
            raise RuntimeError("add after get / get_sum of a key in a client-sharded round "
                               "is not supported (pop the key first)")
        if isinstance(value, RemoteRow):
            self._owner(value.owner)
        else:
            if self.local is None:
                self.local = self.agg._local_entry(self._key, value)
            self.local.add(value, weight)
            self._owner(self.agg.rank)
        self.cur_w = new_w

    def _weighted(self) -> bool:
        return not (self.cur_w is None or self.cur_w == 0)

    def _global_sum(self) -> torch.Tensor:
        """The raw sum over every rank's rows (collective: every rank calls
        it for the same key, as SPMD ``optimize`` does)."""
        if self.sum is not None:
            return self.sum
        local = self.local
        chainable = local is None or getattr(local, "chainable", lambda: True)()
        buf = self.agg._ordered_sum(self.owners, None if local is None else local.partial,
                                    self.P, chainable)
        self.local = None
        self.sum = buf
        return buf

    def _average(self) -> torch.Tensor:
        s = self._global_sum()
        if not self._weighted():
            return s.clone()
        return self.agg.divide(s, self.cur_w)

    def _deliver(self, t: torch.Tensor) -> torch.Tensor:
        return _deliver_to(t.view(self.shape), self.out_device)

    def get(self) -> torch.Tensor:
        return self._deliver(self._average())

    def get_sum(self) -> torch.Tensor:
        return self._deliver(self._global_sum().clone())

    def pop(self, on_device: bool = False) -> torch.Tensor:
        avg = self._average()
        self.sum = None
        return avg.view(self.shape) if on_device else self._deliver(avg)

    def pop_step(self, step: ops.ServerStep) -> None:
        avg = self._average().reshape(-1)
        self.sum = None
        self.agg._apply_step(step, avg)


def _meta(x):
    """The shape / dtype stand-in of a value in the replicated ``add``: the
    reference's arithmetic on meta tensors gives the running sum's promotion,
    broadcasting and errors on every rank without its data (0-dim host
    tensors and Python numbers are themselves)."""
    if isinstance(x, torch.Tensor) and not (x.dim() == 0 and x.device.type == "cpu"):
        return torch.empty(x.shape, dtype=x.dtype, device="meta")
    return x


def _src_type(value) -> Optional[str]:
    """Where an N-d message tensor was produced ("cuda" / "cpu"; a stand-in
    knows its owner's), None for anything else."""
    if isinstance(value, RemoteRow):
        return value.src_type
    if isinstance(value, torch.Tensor) and value.dim() > 0:
        return value.device.type
    return None


def _check_same_device(sum_meta, sum_type: str, value) -> None:
    """The reference's ``sum_v + new_v`` (aggregators.py:38,40) raises for an
    N-d running sum and an N-d value on different devices; the replicated
    meta arithmetic cannot see devices, so every rank checks the recorded
    source types instead and raises together, the key unchanged."""
    vt = _src_type(value)
    if (vt is not None and isinstance(sum_meta, torch.Tensor) and sum_meta.dim() > 0
            and vt != sum_type):
        raise RuntimeError(
            "Expected all tensors to be on the same device: a %s value added to a key "
            "whose running sum is on %s" % (vt, sum_type))


class _ClientShardRef(_TensorEntry):
    """A tensor key of a client-sharded round that keeps the reference's
    arithmetic (aggregators.py:17-40): non-fp32 values (an fp64 / bf16
    model, integer counts), or an fp32 key that stopped fitting the kernel.

    Every rank replays each ``add`` on meta tensors, so all of them know the
    running sum's dtype and shape after every row -- and raise together
    where the reference raises.  A rank keeps ``value * weight`` of its own
    rows (the reference's product, computed at add on the value's device).
    The sum is formed in arrival order through the ranks (the chain in
    either client_reduction mode: the adds of a generic sum are not
    reassociated): rank r receives the running sum of the ranks before it,
    adds its products one by one as the reference does, and passes it on;
    the last holder broadcasts it.  Tensors travel as raw bytes (any dtype,
    gloo or RCCL).  After a get / get_sum the global sum becomes the base
    that later adds continue."""

    def __init__(self, agg: "ClientShardedSerialAggregator", key, base=(0, 0), src_type="cpu"):
        self.agg = agg
        self._key = key
        self.base, self.cur_w = base
        self.meta = _meta(self.base)
        self.rows = []    # this rank's products value * weight, in arrival order
        self.owners = []  # ranks holding rows, in arrival order (one run each)
        self.after = []   # meta of the running sum after each owner's run
        self.dev = agg._reduce_device()
        self.src_type = src_type
        self.out_device = self.dev if src_type == "cuda" else torch.device("cpu")

    def add(self, value, weight) -> None:
        _check_same_device(self.meta, self.src_type, value)
        meta, new_w = reference_add((self.meta, self.cur_w), _meta(value), weight)
        remote = isinstance(value, RemoteRow)
        owner = value.owner if remote else self.agg.rank
        if not (remote or (isinstance(value, torch.Tensor) and value.dim() > 0)):
            # a scalar, held by every rank: it joins the base before any row,
            # else the run of the rank whose rows precede it
            if not self.owners:
                self.base = self.base + (value if weight is None else value * weight)
                self.meta, self.cur_w = _meta(self.base), new_w
                return
            owner = self.owners[-1]
        if owner == self.agg.rank:
            self.rows.append(value if weight is None else value * weight)
        if not self.owners or self.owners[-1] != owner:
            self.owners.append(owner)
            self.after.append(meta)
        else:
            self.after[-1] = meta
        self.meta, self.cur_w = meta, new_w

    def _global_sum(self):
        """Collective: the reference's running sum over every rank's rows."""
        def local(acc):
            for nv in self.rows:
                if isinstance(acc, torch.Tensor) and isinstance(nv, torch.Tensor) and \
                        acc.dim() > 0 and acc.device != nv.device:
                    acc = acc.to(nv.device)
                acc = acc + nv
            return acc

        if self.agg._solo or not self.owners:
            s = local(self.base)
        else:
            s = self.agg._ordered_reference_sum(self.owners, self.after, self.base, local)
        # later adds continue this sum (identical on every rank)
        self.base, self.meta = s, _meta(s)
        self.rows, self.owners, self.after = [], [], []
        return s

    def _deliver(self, t):
        if isinstance(t, torch.Tensor) and t.dim() > 0 and t.device != self.out_device:
            t = _deliver_to(t, self.out_device)
        return t

    def _weighted(self) -> bool:
        return not (self.cur_w is None or self.cur_w == 0)

    def get_sum(self):
        return self._deliver(self._global_sum())

    def get(self):
        s = self._global_sum()
        return self._deliver(reference_quotient(s, self.cur_w) if self._weighted() else s)

    def pop(self, on_device: bool = False):
        return self.get()

    def pop_step(self, step: ops.ServerStep) -> None:
        avg = self.get()
        self.agg._apply_step(step, avg.reshape(-1).to(step.device, torch.float32).contiguous())


class ClientShardedSerialAggregator(SerialAggregator):
    """Client-sharded drop-in for the reference SerialAggregator
    (fedsim/utils/aggregators.py:11-144) for a round loop whose clients are
    split over the ranks of a process group, one process per GPU: each rank
    trains one contiguous block of the round's sampled clients (the
    expensive part of a FedSim round runs N-way parallel) and reduces their
    vectors in HBM; the blocks are then combined with a collective (SURVEY
    §8e, config 5's decomposition on the plugin surface).

    The round driver (CentralFLAlgorithm(..., shard_clients=...)) hands every
    rank every client's message in the reference's arrival order, the
    vectors of other ranks' clients as ``RemoteRow`` stand-ins, so every
    rank runs ``receive_from_client`` for the whole round and keeps the same
    server state (scalar metrics, AdaBest's running statistics, weight sums)
    with the reference's arithmetic.  ``add`` of a stand-in records its
    weight and owner; ``add`` of a local vector goes to this rank's one-GPU
    entry (ring slab / slab rows / borrowed rows, exact order).

    ``get`` / ``get_sum`` / ``pop`` / ``pop_step`` of a tensor key are
    collective (every rank calls them, as the SPMD ``optimize`` does):
      * ``mode="chain"`` (default): the running sum passes from rank to rank
        in arrival order (rank r adds its rows onto rank r-1's sum; N-1
        point-to-point hops of 4P bytes), then the last rank's sum is
        broadcast: every column sums k = 0..K-1 in order, BIT-EXACT;
      * ``mode="allreduce"``: each rank's partial sum from +0, one RCCL
        all-reduce(sum), the divide by fl32(W): reordered, parity normwise
        (<= 1e-6 relative).
    Every rank then applies the server step to its own copy of the cloud
    (same operands, same kernel: same bits), so all ranks hold the new model.

    Args:
        group: the torch.distributed group (default: the default group).
        mode: "chain" or "allreduce".
        entry_factory / step_impl: TEST HOOKS (the per-rank rows and the
            server step on CPU, so the protocol runs over gloo).
        **kwargs: SerialAggregator's options for this rank's rows.
    """

    def __init__(self, group=None, mode: str = "chain", entry_factory: Optional[Callable] = None,
                 step_impl: Optional[Callable] = None, **kwargs) -> None:
        if mode not in ("chain", "allreduce"):
            raise ValueError("mode must be 'chain' or 'allreduce'")
        super().__init__(**kwargs)
        self._group = group
        self._rank, self._world = _group_rank_world(group)
        # one process and no process group: the same round, no collectives
        self._solo = not (dist.is_available() and dist.is_initialized())
        self.mode = mode
        self._entry_factory = entry_factory
        self._step_impl = step_impl

    @property
    def rank(self) -> int:
        return self._rank

    @property
    def world_size(self) -> int:
        return self._world

    @property
    def collective(self) -> bool:
        """Whether this round spans several ranks (collectives run)."""
        return not self._solo

    def client_block(self, n: int):
        """[lo, hi): the positions of the round's n sampled clients this rank
        trains (one contiguous block each, in rank order)."""
        return shard_range(n, self._rank, self._world)

    def _reduce_device(self) -> torch.device:
        if self._entry_factory is not None:
            return torch.device("cpu")
        if self._opts.device is not None:
            return torch.device(self._opts.device)
        return torch.device("cuda", torch.cuda.current_device())

    def _local_entry(self, key, value: torch.Tensor):
        if self._entry_factory is not None:
            return self._entry_factory(value, self)
        dev = self._reduce_device()
        e = _DeviceEntry(value, dev, self._opts, self, out_device=dev)
        if self.mode == "chain":
            # a chained partial continues the previous rank's sum, so no row
            # may be drained from +0 before it: hold every borrowed row (the
            # round's local messages are all alive until received anyway),
            # and grow the ring of snapshotted rows instead of draining it
            e.Bmax = 1 << 62
            e.keep_pending = True
        return e

    # -- collectives shared by the tensor keys and FedDF's teacher targets --
    def _all_true(self, flag: bool) -> bool:
        """Collective AND of a per-rank flag (one int32 all-reduce MIN), so
        every rank takes the same branch -- or raises -- together."""
        if self._solo:
            return bool(flag)
        dev = self._reduce_device()
        if dist.get_backend(self._group) == dist.Backend.GLOO:
            dev = torch.device("cpu")
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._group)
        return bool(t.item())

    def _ordered_sum(self, owners: Sequence[int], local_partial: Optional[Callable], P: int,
                     chainable: bool = True) -> torch.Tensor:
        """Collective: the sum over every rank's rows.  ``owners`` are the
        ranks holding rows, in arrival order (one contiguous run each);
        ``local_partial(acc_in)`` (None when this rank holds no rows) reduces
        this rank's rows in order onto ``acc_in`` (None: from +0).
        chain: rank after rank in ``owners`` order, then a broadcast of the
        last owner's sum (bit-exact arrival order); allreduce: partial sums
        from +0 and one all-reduce(sum) (reordered)."""
        me = self.rank
        if self._solo:
            return local_partial(None)
        if self.mode == "allreduce":
            buf = (local_partial(None) if local_partial is not None
                   else torch.zeros(P, dtype=torch.float32, device=self._reduce_device()))
            _all_reduce_sum(buf, self._group)
            return buf
        if len(set(owners)) != len(owners):
            raise RuntimeError("client_reduction='chain' needs each rank's clients to be one "
                               "contiguous run of the round's arrival order")
        # decided together: a rank that cannot continue the chain (rows
        # already drained from +0) must not leave the others blocked in recv
        if not self._all_true(chainable):
            raise RuntimeError(
                "client_reduction='chain': a rank drained rows of this key from +0 before "
                "the chain reached it (ring full, or host and HBM rows mixed), so the "
                "arrival-order sum cannot be continued bit for bit; raise slab_bytes / "
                "max_rows, or use client_reduction='allreduce'")
        if me in owners:
            i = owners.index(me)
            acc_in = None
            if i > 0:
                acc_in = torch.empty(P, dtype=torch.float32, device=self._reduce_device())
                _recv(acc_in, _global_rank(self._group, owners[i - 1]), self._group)
            buf = local_partial(acc_in)
            if i + 1 < len(owners):
                _send(buf, _global_rank(self._group, owners[i + 1]), self._group)
        else:
            buf = torch.empty(P, dtype=torch.float32, device=self._reduce_device())
        _broadcast(buf, _global_rank(self._group, owners[-1]), self._group)
        return buf

    def _wire_device(self) -> torch.device:
        if dist.get_backend(self._group) == dist.Backend.GLOO:
            return torch.device("cpu")
        return self._reduce_device()

    def _ordered_reference_sum(self, owners, after, base, local):
        """Collective: the running sum of a _ClientShardRef key through the
        ranks in ``owners`` order (``after[i]``: the sum's meta after owner
        i's run; ``local(acc)`` adds this rank's products onto ``acc``), then
        broadcast from the last owner.  Sums travel as raw bytes."""
        if len(set(owners)) != len(owners):
            raise RuntimeError("a client-sharded round needs each rank's clients to be one "
                               "contiguous run of the round's arrival order")
        me, wire = self.rank, self._wire_device()

        def empty_like_meta(m):
            return torch.empty(m.numel() * m.element_size(), dtype=torch.uint8, device=wire)

        def as_bytes(t):
            return t.to(wire).contiguous().reshape(-1).view(torch.uint8)

        def from_bytes(b, m):
            return b.view(m.dtype).reshape(m.shape)

        s = None
        if me in owners:
            i = owners.index(me)
            acc = base
            if i > 0:
                buf = empty_like_meta(after[i - 1])
                _recv(buf, _global_rank(self._group, owners[i - 1]), self._group)
                acc = from_bytes(buf, after[i - 1])
            s = local(acc)
            if i + 1 < len(owners):
                _send(as_bytes(s), _global_rank(self._group, owners[i + 1]), self._group)
        last = after[-1]
        buf = as_bytes(s) if me == owners[-1] else empty_like_meta(last)
        _broadcast(buf, _global_rank(self._group, owners[-1]), self._group)
        return from_bytes(buf, last)

    def divide(self, s: torch.Tensor, W) -> torch.Tensor:
        """fl32(s / fl32(W)), the reference's ``get`` divide."""
        if s.device.type == "cuda":
            return ops.finalize(s, W)
        return s / ops.fl32(W)  # CPU gloo rehearsal: ATen's true divide

    def ordered_rows_sum(self, rows: Optional[torch.Tensor], owners: Sequence[int],
                         n: int) -> torch.Tensor:
        """Collective: the weight-1 sum of every rank's rows ([K_r, n] on rank
        r, None when it holds none), in arrival order under ``chain`` -- the
        reference's ``add(x, 1)`` x K order (FedDF's teacher targets,
        feddf.py:120-126) -- or reordered under ``allreduce``."""
        dev = self._reduce_device()
        local_partial, chainable = None, True
        if rows is not None and rows.shape[0] > 0:
            if self._entry_factory is not None:
                # filled before the chain starts, so its feasibility is part of
                # the collective check (every rank raises together, none waits)
                e = self._entry_factory(rows[0], self)
                for r in rows:
                    e.add(r, 1)
                chainable = getattr(e, "chainable", lambda: True)()
                local_partial = e.partial
            else:
                def local_partial(acc_in):
                    X = rows if rows.device == dev else rows.to(dev)
                    X = X.reshape(X.shape[0], -1).contiguous()
                    out = torch.empty(n, dtype=torch.float32, device=dev)
                    ones = torch.ones(X.shape[0], dtype=torch.float32, device=dev)
                    return ops.reduce_slab(X, ones, out, acc_in=acc_in)
        return self._ordered_sum(owners, local_partial, n, chainable)

    def broadcast_from(self, t: torch.Tensor, src: int) -> torch.Tensor:
        """Collective: ``t`` on rank ``src`` copied into ``t`` on every rank
        (a host tensor under RCCL travels through this rank's GPU)."""
        if self._solo:
            return t
        if t.device.type == "cpu" and dist.get_backend(self._group) != dist.Backend.GLOO:
            d = t.to(self._reduce_device())
            _broadcast(d, _global_rank(self._group, src), self._group)
            t.copy_(d)
            return t
        _broadcast(t, _global_rank(self._group, src), self._group)
        return t

    def _apply_step(self, step: ops.ServerStep, avg: torch.Tensor) -> None:
        if self._step_impl is not None:
            self._step_impl(step, avg)
        else:
            step.apply(avg if avg.device == step.device else avg.to(step.device))

    def add(self, key, value, weight=None):
        """Every rank makes the same choice (the values' dtypes and shapes
        and the weights are known everywhere): fp32 tensors with real
        weights go to the exact HIP rows (_ClientShardEntry); anything else
        keeps the reference's arithmetic (_ClientShardRef), continuing a
        kernel key's exact sum when a value stops fitting it."""
        e = self._members.get(key)
        tensor = isinstance(value, torch.Tensor) and value.dim() > 0
        if not tensor and not isinstance(e, _TensorEntry):
            super().add(key, value, weight)  # scalar key: the host arithmetic
            return
        src = value.src_type if isinstance(value, RemoteRow) else \
            value.device.type if tensor else "cpu"
        if isinstance(e, _ClientShardEntry) and _kernel_value(value, weight) and \
                tuple(value.shape) == e.shape and src == e.src_type:
            e.add(value, weight)
            return
        if isinstance(e, _ClientShardEntry) and tensor and src != e.src_type:
            # the reference's sum_v + new_v raises; the key stays as it was
            _check_same_device(torch.empty(e.shape, device="meta"), e.src_type, value)
        if e is None and _kernel_value(value, weight):
            e = _ClientShardEntry(self, value.shape, src)
            e._key = key
            e.add(value, weight)  # may raise (weight None): the key is not created
            self._members[key] = e
            return
        if isinstance(e, _ClientShardEntry):
            # leave the kernel: the exact sum so far (collective, every rank
            # reaches this add) is the base of the reference arithmetic
            e = self._members[key] = _ClientShardRef(self, key, (e.get_sum(), e.cur_w),
                                                     src_type=e.src_type)
        if isinstance(e, _ClientShardRef):
            e.add(value, weight)  # raises as the reference's add would
            return
        r = _ClientShardRef(self, key, e if e is not None else (0, 0), src_type=src)
        r.add(value, weight)  # may raise: the key stays as it was
        self._members[key] = r

    def exchange(self, local_msgs: dict, n: int, failed: bool = False, extras=None):
        """Every rank's client messages of this round, position by position:
        this rank's own as given, the others' rebuilt from what their ranks
        sent (tensors as RemoteRow stand-ins, 0-dim tensors and everything
        else by value).  Collective.  ``failed``: this rank's clients raised;
        every rank then gets None (and raises), none is left waiting.
        ``extras``: any picklable per-rank value; with it, returns
        ``(messages, [extras of rank 0, 1, ...])``."""
        if self._solo:
            msgs = None if failed else [None] * n
            return msgs if extras is None else (msgs, [extras])
        mine = None if failed else {p: _skeleton(m, self._rank) for p, m in local_msgs.items()}
        every = [None] * self._world
        dist.all_gather_object(every, (mine, extras), group=self._group)
        got = [e[1] for e in every]
        if any(e[0] is None for e in every):
            return None if extras is None else (None, got)
        dev = self._reduce_device()
        out = [None] * n
        for r, (msgs, _) in enumerate(every):
            if r == self._rank:
                continue
            for p, m in msgs.items():
                out[p] = _flesh(m, dev)
        return out if extras is None else (out, got)

    def reserve(self, key, P, device):
        """No reserved rows: a rank trains all its clients before any of them
        is received, and a ring hands out one row at a time; the clients'
        fresh vectors are borrowed at ``add`` instead (no copy)."""
        return None
