"""Scripted SerialAggregator sessions over non-fp32 / mixed-type keys.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  One list of scenarios,
replayed identically by tools/gen_golden_generic.py (through the REFERENCE's
own SerialAggregator, fedsim/utils/aggregators.py:11-144, imported in the
build container) and by tests/test_generic_keys.py / tests/test_gpu_generic_
keys.py (through fedsim_amd's drop-in and oracle/reference_loop's
restatement).  Every result -- tensors as raw bytes + dtype + shape, Python
numbers exactly, exceptions by type -- goes into one transcript; two
transcripts are equal iff every get / get_sum / get_weight / pop / pop_all
returned the same bits.

A scenario is a list of steps:
  ("add", key, value, weight)   value: a ValueSpec (a tensor built from
                                oracle/vectors) or a Python number
  ("get" | "get_sum" | "get_weight" | "pop", key)
  ("pop_all",) | ("keys",) | ("in", key)
"""
from __future__ import annotations

import base64
from typing import Dict, List

import numpy as np
import torch

from . import vectors as V

_DTYPES = {
    "f64": torch.float64, "f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16,
    "i64": torch.int64, "i32": torch.int32, "i16": torch.int16, "u8": torch.uint8,
    "bool": torch.bool,
}


class ValueSpec(object):
    """A deterministic tensor: ``dtype`` ("f64", "bf16", ...), ``shape``,
    ``seed``; floats are gauss * scale, integers uniform in [lo, hi]."""

    __slots__ = ("dtype", "shape", "seed", "scale", "lo", "hi")

    def __init__(self, dtype, shape, seed, scale=1.0, lo=-1000, hi=1000):
        self.dtype, self.shape, self.seed = dtype, tuple(shape), seed
        self.scale, self.lo, self.hi = scale, lo, hi

    def build(self) -> torch.Tensor:
        n = int(np.prod(self.shape)) if self.shape else 1
        dt = _DTYPES[self.dtype]
        if dt.is_floating_point:
            t = torch.from_numpy(V.gauss(self.seed, n) * self.scale).to(dt)
        elif dt == torch.bool:
            t = torch.from_numpy(V.randint(self.seed, n, 0, 1)).to(dt)
        else:
            t = torch.from_numpy(V.randint(self.seed, n, self.lo, self.hi)).to(dt)
        return t.reshape(self.shape)

    def __repr__(self):
        return f"{self.dtype}{list(self.shape)}#{self.seed}"


def S(dtype, shape, seed, **kw) -> ValueSpec:
    return ValueSpec(dtype, shape, seed, **kw)


def _adds(key, specs, weights):
    return [("add", key, s, w) for s, w in zip(specs, weights)]


def _reads(key):
    return [("get_weight", key), ("get_sum", key), ("get", key)]


P = 1031  # odd: the f64 finalize kernel's scalar tail and f32x4 tails run


def scenarios() -> Dict[str, List[tuple]]:
    sc = {}
    w5 = [37, 12.5, 400, 3, 0.1]
    for dt in ("f64", "bf16", "f16"):
        specs = [S(dt, (P,), 100 + i, scale=0.3) for i in range(5)]
        sc[f"{dt}_weighted"] = _adds("p", specs[:2], w5[:2]) + _reads("p") + \
            _adds("p", specs[2:], w5[2:]) + _reads("p") + [("pop", "p"), ("in", "p")]
        sc[f"{dt}_matrix_int_weights"] = _adds("m", [S(dt, (7, 33), 150 + i) for i in range(4)],
                                              [5, 9, 1, 60]) + [("pop", "m")]
    # integers: exact sums, true division into the default float dtype
    sc["i64_int_weights"] = _adds("c", [S("i64", (P,), 200 + i) for i in range(4)],
                                  [3, 8, 1, 5]) + _reads("c") + [("pop", "c")]
    sc["i64_float_weights"] = _adds("c", [S("i64", (P,), 210 + i, lo=-10**6, hi=10**6)
                                          for i in range(3)], [0.5, 2.25, 7.3]) + \
        [("pop", "c")]
    sc["i32_zero_total_weight"] = _adds("z", [S("i32", (64,), 220), S("i32", (64,), 221)],
                                        [2, -2]) + _reads("z") + [("pop", "z")]
    sc["bool_counts"] = _adds("b", [S("bool", (99,), 230 + i) for i in range(3)], [1, 1, 1]) + \
        [("pop", "b")]
    sc["u8_counts"] = _adds("u", [S("u8", (40,), 235 + i, lo=0, hi=255) for i in range(3)],
                            [1, 2, 3]) + [("pop", "u")]
    sc["f64_zero_weight_first"] = _adds("q", [S("f64", (P,), 240), S("f64", (P,), 241)],
                                        [0, 4]) + _reads("q") + [("pop", "q")]
    # promotion across adds (the running sum changes dtype as torch's rules say)
    sc["f32_then_f64"] = _adds("p", [S("f32", (P,), 300), S("f32", (P,), 301),
                                     S("f64", (P,), 302)], [3, 5, 2.5]) + _reads("p") + \
        [("pop", "p")]
    sc["f64_then_f32"] = _adds("p", [S("f64", (P,), 310), S("f32", (P,), 311)], [3, 5]) + \
        [("pop", "p")]
    sc["f32_then_bf16"] = _adds("p", [S("f32", (P,), 320), S("bf16", (P,), 321),
                                      S("f32", (P,), 322)], [3, 5, 7]) + [("pop", "p")]
    sc["bf16_then_f32"] = _adds("p", [S("bf16", (P,), 330), S("f32", (P,), 331)], [3, 5]) + \
        [("pop", "p")]
    sc["i64_then_f32"] = _adds("p", [S("i64", (P,), 340), S("f32", (P,), 341)], [3, 5]) + \
        [("pop", "p")]
    sc["f32_then_i64"] = _adds("p", [S("f32", (P,), 345), S("i64", (P,), 346)], [3, 5]) + \
        [("pop", "p")]
    # scalars meeting tensors (broadcast), shape changes (broadcast)
    sc["scalar_then_tensor"] = [("add", "s", 0.5, 2), ("add", "s", S("f32", (P,), 350), 3),
                                ("pop", "s")]
    sc["tensor_then_scalar"] = [("add", "s", S("f32", (P,), 355), 3), ("add", "s", 1.25, 2)] + \
        _reads("s") + [("pop", "s")]
    sc["tensor_then_0dim"] = [("add", "s", S("f64", (P,), 357), 3),
                              ("add", "s", S("f64", (), 358), 2), ("pop", "s")]
    sc["broadcast_row"] = [("add", "r", S("f32", (5, 16), 360), 2),
                           ("add", "r", S("f32", (16,), 361), 3), ("pop", "r")]
    sc["f32_tensor_0dim_weight"] = [("add", "t", S("f32", (P,), 365), S("f64", (), 366)),
                                    ("add", "t", S("f32", (P,), 367), S("i64", (), 368, lo=1,
                                                                        hi=9))] + \
        _reads("t") + [("pop", "t")]
    # errors: the reference raises, the key is left as it was
    sc["weight_none_errors"] = [("add", "e", S("f64", (P,), 370), None), ("in", "e"),
                                ("add", "e", S("f64", (P,), 371), 2),
                                ("add", "e", S("f64", (P,), 372), None), ("pop", "e")]
    sc["shape_mismatch_errors"] = [("add", "x", S("f64", (8,), 380), 1),
                                   ("add", "x", S("f64", (9,), 381), 1), ("get", "x"),
                                   ("add", "y", S("f32", (8,), 382), 1),
                                   ("add", "y", S("f32", (9,), 383), 1), ("pop", "y"),
                                   ("pop", "x")]
    sc["missing_key_errors"] = [("get", "nope"), ("get_sum", "nope"), ("get_weight", "nope"),
                                ("pop", "nope")]
    # a whole round's worth of mixed keys, read back with pop_all
    sc["mixed_pop_all"] = [("add", "local_params", S("f64", (P,), 390), 37),
                           ("add", "clients.train.loss", 0.75, 37),
                           ("add", "counts", S("i64", (10,), 391, lo=0, hi=50), 1),
                           ("add", "local_params", S("f64", (P,), 392), 12),
                           ("add", "clients.train.loss", 0.5, 12),
                           ("add", "counts", S("i64", (10,), 393, lo=0, hi=50), 1),
                           ("add", "half", S("bf16", (3, 11), 394), 0.25),
                           ("keys",), ("pop_all",), ("keys",)]
    return sc


def n_tensor_adds(steps) -> int:
    return sum(1 for s in steps if s[0] == "add" and isinstance(s[2], ValueSpec)
               and len(s[2].shape) > 0)


def needs_kernel(steps) -> bool:
    """Whether a scenario starts a key on the HIP kernel path (an fp32 N-d
    tensor as a key's first value): on a host without a GPU fedsim_amd
    raises for those, by design.  A key that starts as anything else keeps
    the reference's arithmetic whatever is added to it later."""
    started = set()
    for s in steps:
        if s[0] == "pop_all":
            started.clear()
        if s[0] == "pop":
            started.discard(s[1])
        if s[0] != "add" or s[1] in started:
            continue
        started.add(s[1])
        if isinstance(s[2], ValueSpec) and s[2].dtype == "f32" and len(s[2].shape) > 0:
            return True
    return False


# -- transcripts ------------------------------------------------------------
def encode(x):
    """A result as a JSON-able, bit-exact record."""
    if isinstance(x, torch.Tensor):
        t = x.detach().cpu().contiguous()
        raw = t.reshape(-1).view(torch.uint8).numpy().tobytes()
        return {"t": str(t.dtype).replace("torch.", ""), "shape": list(t.shape),
                "b64": base64.b64encode(raw).decode()}
    if isinstance(x, bool) or x is None:
        return {"v": x}
    if isinstance(x, int):
        return {"i": str(x)}
    if isinstance(x, float):
        return {"f": x.hex()}
    if isinstance(x, dict):
        return {"d": [[k, encode(v)] for k, v in x.items()]}
    if isinstance(x, (list, tuple)):
        return {"l": [encode(v) for v in x]}
    return {"repr": repr(x)}


def replay(agg, steps, device=None, wrap=None) -> list:
    """Run ``steps`` on ``agg`` (tensor values moved to ``device`` when given)
    and return the transcript.  ``wrap(j, t)``: what the j-th N-d tensor
    value of the scenario is handed over as (a client-sharded round passes
    another rank's vectors as stand-ins)."""
    out = []
    j = 0
    for st in steps:
        op = st[0]
        try:
            if op == "add":
                _, key, value, weight = st
                if isinstance(value, ValueSpec):
                    value = value.build()
                    if device is not None:
                        value = value.to(device)
                    if wrap is not None and value.dim() > 0:
                        value = wrap(j, value)
                        j += 1
                if isinstance(weight, ValueSpec):
                    weight = weight.build()  # 0-dim host tensor weights stay on the host
                agg.add(key, value, weight)
                res = None
            elif op in ("get", "get_sum", "get_weight", "pop"):
                res = getattr(agg, op)(st[1])
            elif op == "pop_all":
                res = agg.pop_all()
            elif op == "keys":
                res = list(agg.keys())
            elif op == "in":
                res = st[1] in agg
            else:
                raise ValueError(op)
            out.append(["ok", encode(res)])
        except Exception as e:  # noqa: BLE001 -- the transcript records what was raised
            out.append(["raise", type(e).__name__])
    return out
