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

The per-rank reduction is the HIP kernel (``ops.reduce_slab``); ``local_reduce``
can be injected so the host-side protocol is testable with gloo on CPU.
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


def _hip_reduce(X, w32, out, acc_in=None, W=None, flags=0):
    return ops.reduce_slab(X, w32, out, acc_in=acc_in, W=W, P=out.numel(), flags=flags)


def param_sharded(X_shard: torch.Tensor, w32: torch.Tensor, W, out_shard: torch.Tensor,
                  local_reduce: Callable = _hip_reduce, flags: int = 0) -> torch.Tensor:
    """Reduce this rank's column shard of all K clients (no collective)."""
    return local_reduce(X_shard, w32, out_shard, None, W, flags)


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
