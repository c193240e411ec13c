"""ctypes binding of the C oracle (fedagg_ref.c) plus a numpy twin.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Host-side semantics the oracle also restates (pure Python, as the reference):
  * weight of a client: ``train_weight`` or ``num_samples[train]``
    (fedsim/distributed/centralized/training/utils.py:42-43); clients with
    weight <= 0 are skipped (utils.py:45); a diverged client aborts (utils.py:39-40)
  * total weight W: the Python running sum ``cur_w + new_w``
    (fedsim/utils/aggregators.py:40) — int for FedAvg, float for FedNova
  * rounding of a Python scalar against an fp32 tensor: fl32(scalar)
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfedagg_ref.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
        os.path.join(_HERE, "fedagg_ref.c")
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, f32, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int
        L.ref_reduce_f32.argtypes = [vp, i64, vp, i64, i64, vp, vp, f32, ci]
        L.ref_finalize_f32.argtypes = [vp, f32, i64, vp]
        L.ref_fedavg_sgd_f32.argtypes = [vp, f32, vp, vp, i64]
        L.ref_adabest_sgd_f32.argtypes = [vp, f32, f32, vp, vp, vp, i64]
        L.ref_feddyn_sgd_f32.argtypes = [vp, f32, f32, vp, vp, vp, vp, i64]
        L.ref_server_step_f32.argtypes = [ci, vp, f32, vp, vp, vp, vp, ci, vp, f32, f32, f32,
                                          f32, ci, ci, i64]
        L.ref_teacher_linear_f32.argtypes = [vp, i64, vp, i64, i64, i64, i64, i64, i64, i64,
                                             vp, ci]
        L.ref_teacher_conv2d_f32.argtypes = [vp, i64, vp, i64, i64, i64, i64] + [i64] * 13 + [
            vp, ci, i64]
        L.ref_pad_lrn_maxpool_f32.argtypes = [vp] + [i64] * 9 + [f32] * 3 + [i64] * 6 + [vp]
        for fn in ("ref_reduce_f32", "ref_finalize_f32", "ref_fedavg_sgd_f32",
                   "ref_adabest_sgd_f32", "ref_feddyn_sgd_f32", "ref_server_step_f32",
                   "ref_teacher_linear_f32", "ref_teacher_conv2d_f32", "ref_pad_lrn_maxpool_f32"):
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def fl32(x) -> np.float32:
    return np.float32(x)


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def accepted(weights: Sequence, diverged: Optional[Sequence[bool]] = None):
    """Indices and weights the reference adds, plus the round status.

    Returns (idx, w, W, ok): ok is False if a diverged client aborted the round
    (centralized_fl_algorithm.py:427-432); W is the Python running sum or None
    when no client had weight > 0 (then "local_params" is not in the aggregator).
    """
    idx, ws, W = [], [], 0
    for k, w in enumerate(weights):
        if diverged is not None and diverged[k]:
            return idx, ws, (W if idx else None), False
        if w > 0:
            idx.append(k)
            ws.append(w)
            W = W + w
    return idx, ws, (W if idx else None), True


def reduce(X: np.ndarray, weights: Sequence, acc_in: Optional[np.ndarray] = None,
           W=None) -> np.ndarray:
    """C oracle: weighted sequential reduce of rows of X ([B, P] fp32)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    B, P = X.shape
    w32 = np.array([fl32(w) for w in weights], dtype=np.float32)
    out = np.empty(P, dtype=np.float32)
    lib().ref_reduce_f32(_p(X), P, _p(w32), B, P, _p(acc_in), _p(out),
                         float(fl32(W)) if W is not None else 0.0, 1 if W is not None else 0)
    return out


def finalize(acc: np.ndarray, W) -> np.ndarray:
    acc = np.ascontiguousarray(acc, dtype=np.float32)
    out = np.empty_like(acc)
    lib().ref_finalize_f32(_p(acc), float(fl32(W)), acc.size, _p(out))
    return out


def fedavg_sgd(avg: np.ndarray, cloud: np.ndarray, lr: float) -> np.ndarray:
    c = np.array(cloud, dtype=np.float32, copy=True)
    a = np.ascontiguousarray(avg, dtype=np.float32)
    lib().ref_fedavg_sgd_f32(_p(a), float(fl32(lr)), _p(c), None, c.size)
    return c


def adabest_sgd(avg: np.ndarray, cloud: np.ndarray, avg_prev: np.ndarray, beta: float,
                lr: float):
    c = np.array(cloud, dtype=np.float32, copy=True)
    ap = np.array(avg_prev, dtype=np.float32, copy=True)
    a = np.ascontiguousarray(avg, dtype=np.float32)
    lib().ref_adabest_sgd_f32(_p(a), float(fl32(beta)), float(fl32(lr)), _p(c), _p(ap), None,
                              c.size)
    return c, ap


def feddyn_sgd(avg: np.ndarray, cloud: np.ndarray, h: np.ndarray, weight, num_clients,
               lr: float):
    """Returns (cloud', h', avg_params')."""
    c = np.array(cloud, dtype=np.float32, copy=True)
    hh = np.array(h, dtype=np.float32, copy=True)
    a = np.ascontiguousarray(avg, dtype=np.float32)
    ap = np.empty_like(c)
    lib().ref_feddyn_sgd_f32(_p(a), float(fl32(weight / num_clients)), float(fl32(lr)), _p(c),
                             _p(hh), _p(ap), None, c.size)
    return c, hh, ap


class ServerState(object):
    """Oracle-side server state across rounds: cloud, the SGD momentum buffer
    and the algorithm's auxiliary vector (AdaBest avg_params / FedDyn h)."""

    ALGO = {"fedavg": 0, "adabest": 1, "feddyn": 2}

    def __init__(self, algo, cloud, opt, aux=None, coef=0.0):
        self.algo = algo
        self.cloud = np.array(cloud, dtype=np.float32, copy=True)
        self.opt = dict(opt)
        self.aux = None if aux is None else np.array(aux, dtype=np.float32, copy=True)
        self.coef = coef
        self.buf = None
        self.grad = None
        self.avg_prev = None

    def step(self, avg):
        o = self.opt
        P = self.cloud.size
        mom = o.get("momentum", 0.0)
        init = self.buf is None
        if mom and init:
            self.buf = np.empty(P, dtype=np.float32)
        self.grad = np.empty(P, dtype=np.float32)
        self.avg_prev = np.empty(P, dtype=np.float32) if self.algo == "feddyn" else None
        a = np.ascontiguousarray(avg, dtype=np.float32)
        lib().ref_server_step_f32(
            self.ALGO[self.algo], _p(a), float(fl32(self.coef)), _p(self.cloud), _p(self.aux),
            _p(self.avg_prev), _p(self.buf), int(init), _p(self.grad),
            float(fl32(-o["lr"])), float(fl32(mom)), float(fl32(1 - o.get("dampening", 0.0))),
            float(fl32(o.get("weight_decay", 0.0))), int(o.get("nesterov", False)),
            int(o.get("maximize", False)), P)


# ---- numpy twin (independent restatement of the reduce / divide) ----------

def reduce_numpy(X: np.ndarray, weights: Sequence) -> np.ndarray:
    acc = np.zeros(X.shape[1], dtype=np.float32)
    for k in range(X.shape[0]):
        prod = X[k].astype(np.float32) * np.float32(weights[k])
        acc = acc + prod
    return acc


def finalize_numpy(acc: np.ndarray, W) -> np.ndarray:
    return (acc / np.float32(W)).astype(np.float32)


def teacher_linear(x: np.ndarray, slab: np.ndarray, w_off: int, b_off: int, in_f: int,
                   out_f: int, shared: bool, relu: bool = False) -> np.ndarray:
    """C oracle of fedagg_teacher_linear_f32 (an f32 fmaf chain in input
    order; see fedagg_ref.c)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    slab = np.ascontiguousarray(slab, dtype=np.float32)
    K, P = slab.shape
    M = x.size // in_f if shared else x.size // (in_f * K)
    y = np.empty((K, M, out_f), dtype=np.float32)
    lib().ref_teacher_linear_f32(_p(x), 0 if shared else M * in_f, _p(slab), P, w_off, b_off,
                                 K, M, in_f, out_f, _p(y), int(relu))
    return y


def teacher_conv2d(x: np.ndarray, slab: np.ndarray, w_off: int, b_off: int, out_channels: int,
                   kernel_size, stride, padding, shared: bool, relu: bool = False,
                   cc: int = 0) -> np.ndarray:
    """C oracle of fedagg_teacher_conv2d_f32 (the fmaf chain over
    (c, kh, kw) in order, or, cc > 0, the LDS-resident kernel's chunked order
    that fedagg_conv_order reports; see fedagg_ref.c).  padding = (top,
    bottom, left, right); returns [K, M, OC, OH, OW]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    slab = np.ascontiguousarray(slab, dtype=np.float32)
    K, P = slab.shape
    M, C, H, W = x.shape[-4:]
    KH, KW = kernel_size
    sh, sw = stride
    pt, pb, pl, pr = padding
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    y = np.empty((K, M, out_channels, OH, OW), dtype=np.float32)
    lib().ref_teacher_conv2d_f32(_p(x), 0 if shared else M * C * H * W, _p(slab), P, w_off, b_off,
                                 K, M, C, H, W, out_channels, KH, KW, sh, sw, pt, pl, OH, OW,
                                 _p(y), int(relu), int(cc))
    return y


def pad_lrn_maxpool(x: np.ndarray, pads=(0, 0, 0, 0), lrn=None, pool=None) -> np.ndarray:
    """C oracle of fedagg_pad_lrn_maxpool_f32 over the last three dimensions
    (C, H, W) of x: zero pads (top, bottom, left, right), lrn (size, alpha,
    beta, k) or None, pool (kh, kw, sh, sw, ph, pw) or None."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    C, H, W = x.shape[-3:]
    N = x.size // (C * H * W) if x.size else 0
    size, alpha, beta, k = lrn if lrn is not None else (0, 0.0, 0.0, 0.0)
    kh, kw, sh, sw, ph, pw = pool if pool is not None else (0, 0, 0, 0, 0, 0)
    Hp, Wp = H + pads[0] + pads[1], W + pads[2] + pads[3]
    if kh == 0:
        OH, OW = Hp, Wp
    else:
        OH, OW = (Hp + 2 * ph - kh) // sh + 1, (Wp + 2 * pw - kw) // sw + 1
    y = np.empty((*x.shape[:-2], OH, OW), dtype=np.float32)
    lib().ref_pad_lrn_maxpool_f32(_p(x), N, C, H, W, *pads, size, alpha, beta, k, kh, kw, sh, sw,
                                  ph, pw, _p(y))
    return y
