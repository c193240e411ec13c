"""Flat-vector <-> module parameter conversion (the pack / unpack edges of the
path).  Layout = concatenation of ``module.parameters()`` in registration order,
each parameter's row-major storage (reference: fedsim/utils/convert_parameters.py:78-94,
129-148)."""
from __future__ import annotations

from collections import OrderedDict

import torch
from torch import Tensor

from .. import ops
from torch.nn import Module
from torch.nn.utils import parameters_to_vector, vector_to_parameters


def vector_to_parameters_like(vec: Tensor, parameters_like):
    """Views of ``vec`` shaped like each of ``parameters_like`` (no copy)."""
    if not isinstance(vec, torch.Tensor):
        raise TypeError("expected torch.Tensor, but got: {}".format(torch.typename(vec)))
    out, ptr = [], 0
    for p in parameters_like:
        n = p.numel()
        out.append(vec[ptr: ptr + n].view_as(p).data)
        ptr += n
    return out


def vector_to_named_parameters_like(vec: Tensor, named_parameters_like) -> OrderedDict:
    if not isinstance(vec, torch.Tensor):
        raise TypeError("expected torch.Tensor, but got: {}".format(torch.typename(vec)))
    out, ptr = OrderedDict(), 0
    for key, p in named_parameters_like:
        n = p.numel()
        out[key] = vec[ptr: ptr + n].view_as(p)
        ptr += n
    return out


def vectorize_module(module: Module, clone=True, detach=True, out=None) -> Tensor:
    """``module``'s parameters as one flat vector (reference:
    fedsim/utils/convert_parameters.py:78-94).

    The reference's ``clone`` is a second copy of what ``parameters_to_vector``
    (``torch.cat``) has just written to fresh memory: the result already
    shares nothing with the parameters, so the copy is skipped and the
    returned vector is the same either way.

    ``out``: a reserved slab row (slab_rows.SlabRow, from
    ``slab_rows.reserve_round_row``): the parameters are written straight into
    it (fedagg_pack_segments_f32, one launch) and the row is returned."""
    if out is not None:
        from .slab_rows import SlabRow

        if not isinstance(out, SlabRow) or not out.in_slab:
            raise TypeError("out must be a reserved SlabRow still in its slab")
        if out._committed:  # its contents are the aggregator's now
            raise ValueError("out was already added to the aggregator; reserve a new row")
        params = [p.detach() for p in module.parameters()]
        P = sum(p.numel() for p in params)
        if P != out.shape[0]:
            raise ValueError(f"module has {P} parameters, the row {out.shape[0]}")
        ops.pack_segments(params, out._slab, out._row)
        return out
    vec = parameters_to_vector(module.parameters())
    if detach:
        vec = vec.detach()
    return vec


def initialize_module(module: Module, vec: Tensor, clone=True, detach=True) -> bool:
    if clone:
        vec = vec.clone()
    if detach:
        vec = vec.detach()
    if sum(p.numel() for p in module.parameters()) != vec.numel():
        return False
    vector_to_parameters(vec, module.parameters())
    return True


def vectorize_module_grads(module: Module, clone=True, detach=True):
    """Gradients of ``module.parameters()`` packed like ``vectorize_module``
    (reference: convert_parameters.py:97-126); None if any parameter has no
    gradient yet.  Parameters on different devices raise TypeError, as
    torch's parameters_to_vector does."""
    grads = []
    for p in module.parameters():
        if p.grad is None:
            return None
        grads.append(p.grad)
    if grads and any(g.device != grads[0].device for g in grads):
        raise TypeError("Found two parameters on different devices, this is currently "
                        "not supported.")
    vec = torch.cat([g.reshape(-1) for g in grads]) if grads else torch.empty(0)
    if clone:
        vec = vec.clone()
    if detach:
        vec = vec.detach()
    return vec
