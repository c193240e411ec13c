"""Explicit hand-over of client vectors inside the round driver.

The reference snapshots every client vector at receive
(``local_params.clone().detach().data``, fedsim/distributed/centralized/
training/utils.py:34).  The round driver's aggregator can instead read an
HBM vector in place (``borrow``) or stage a host vector after ``add``
returns (``borrow_host``) -- sound only when the client gave the vector
away: it keeps no reference or view and will not change it.

Ownership is declared, not inferred.  The producer of a client message
calls ``hand_over(t)`` on the vector it returns (the library's clients do,
local_updates.py; a user ``send_to_server`` may); the round driver opens a
``handover_round()`` per round, and ``serial_aggregation`` accepts a vector
as handed over only if

* it carries a token of the open round: the same tensor object, at the same
  version (unchanged since it was handed over);
* no other tensor shares its storage (a view kept by the client, or the
  base it is a view of: ``_base`` / the storage's use count);
* no earlier vector of the round was handed over from the same storage.

A row the client reserved in the round's slab (``reserve_round_row`` +
``vectorize_module(out=row)``) is handed over by that protocol: it is the
aggregator's memory, a committed row cannot be written again, and torch ops
on the SlabRow act on a private copy.  Anything else -- a vector without a
token (a user client that did not declare it), a changed one, an aliased one
-- gets the reference's clone.
A producer that calls ``hand_over`` and still changes the very tensor in
place before the round is reduced breaks its declaration: the version
counter makes that reduction raise instead of reading changed data.

Outside a hand-over round (``receive_from_client`` called by user code) no
token exists: nothing is handed over and a borrowing aggregator gets the
reference's clone.  User code that wants the borrow declares it the same way:
``with handover_round(): ... hand_over(v) ...``.
"""
from __future__ import annotations

import weakref
from contextlib import contextmanager
from typing import Optional

import torch

from .slab_rows import SlabRow

__all__ = ["hand_over", "handover_round", "take_token", "unaliased"]


class _Round(object):
    __slots__ = ("tokens", "storages")

    def __init__(self):
        self.tokens = {}      # id(t) -> (weakref(t), version at hand-over)
        self.storages = set()  # storages of the vectors accepted this round


_OPEN = []  # the driver's open rounds (nested drivers: innermost last)


def hand_over(t):
    """Declare that ``t`` is given away to the server (see the module
    docstring); returns ``t``.  A no-op outside a driver round.

    What is detected afterwards is torch's version counter: an in-place
    torch op on ``t`` (or a view of it) between this call and the read
    makes the reduction raise.  Writes that bypass the counter are NOT
    detected -- ``t.data.copy_(...)``, writes through ``t.numpy()`` or a
    DLPack / ``__array_interface__`` alias, or a kernel writing the storage
    by pointer -- and the aggregator then reads the changed values.  A
    producer that keeps a handle it may write that way must not hand the
    tensor over (only the library's own ``sgd_update`` calls this today)."""
    if _OPEN and isinstance(t, torch.Tensor):
        _OPEN[-1].tokens[id(t)] = (weakref.ref(t), t._version)
    return t


@contextmanager
def handover_round():
    """The scope of one round of the driver: tokens live until it closes."""
    _OPEN.append(_Round())
    try:
        yield
    finally:
        _OPEN.pop()


def take_token(t) -> Optional[bool]:
    """None outside a hand-over round (nothing was declared); else whether
    ``t`` carries a valid token of the open round (consumed) and its storage
    was not handed over before in this round."""
    if not _OPEN:
        return None
    rnd = _OPEN[-1]
    tok = rnd.tokens.pop(id(t), None)
    if tok is None or tok[0]() is not t or t._version != tok[1]:
        return False
    key = _storage_key(t)
    if key in rnd.storages:
        return False
    rnd.storages.add(key)
    return True


def _storage_key(t):
    dense = getattr(t, "_dense", None)
    if dense is not None:  # a SlabRow read back into its own copy
        t = dense
    try:
        return (t.device, t.untyped_storage().data_ptr())
    except (RuntimeError, NotImplementedError):
        return (t.device, id(t))


def unaliased(t) -> bool:
    """No other tensor (view, base, alias) shares ``t``'s storage: one
    TensorImpl on it plus the temporary storage object made here."""
    if not isinstance(t, torch.Tensor) or t._base is not None:
        return False
    if isinstance(t, SlabRow):
        if t.in_slab:  # a reserved slab row: no storage of its own
            return True
        # read back already: torch ops on it may have handed out views of
        # its copy, which add would then borrow
        t = t._dense
        if t is None:
            return False
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata) <= 2
