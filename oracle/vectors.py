"""Deterministic, platform-independent test inputs for the aggregation path.

TEST INFRASTRUCTURE (oracle/): only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this package.

Inputs are built from a splitmix64 counter hash with integer arithmetic and
exact float64 sums only (no libm calls), so every platform regenerates them bit
for bit; the golden manifest also stores a SHA-256 of every regenerated input
so any drift is caught instead of showing up as a parity failure.
"""
from __future__ import annotations

import hashlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform01(seed: int, n: int) -> np.ndarray:
    """n float64 values in [0, 1), exact multiples of 2**-53."""
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x100000001B3)
    h = _splitmix64(_splitmix64(ctr) ^ np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def gauss(seed: int, n: int) -> np.ndarray:
    """Irwin-Hall(4) approximation of N(0, 1): mean 0, variance 1, float64."""
    s = (uniform01(seed * 4 + 0, n) + uniform01(seed * 4 + 1, n)) + (
        uniform01(seed * 4 + 2, n) + uniform01(seed * 4 + 3, n)
    )
    return (s - 2.0) * 1.7320508075688772


def randint(seed: int, n: int, lo: int, hi: int) -> np.ndarray:
    """n integers uniform in [lo, hi] (inclusive)."""
    u = uniform01(seed, n)
    return lo + np.floor(u * (hi - lo + 1)).astype(np.int64)


def client_rows(dist: str, K: int, P: int, seed: int) -> np.ndarray:
    """[K, P] fp32 client parameter vectors.

    normal     x ~ N(0, 1)                     (cancelling sums)
    realistic  x = base + eps_k, base ~ N(0, 0.05), eps_k ~ N(0, 1e-3)
               (clients that all started from the same global model)
    special    realistic values with +-0.0, subnormals and large magnitudes
               mixed in (kept finite through the reduction: no NaN payloads)
    """
    if dist == "normal":
        return np.stack([gauss(seed * 100003 + k, P) for k in range(K)]).astype(np.float32)
    base = 0.05 * gauss(seed * 7919 + 7, P)
    X = np.stack([base + 1e-3 * gauss(seed * 100003 + k, P) for k in range(K)])
    if dist == "realistic":
        return X.astype(np.float32)
    if dist == "special":
        X = X.astype(np.float32)
        sel = uniform01(seed * 31 + 5, K * P).reshape(K, P)
        X[sel < 0.05] = np.float32(-0.0)
        X[(sel >= 0.05) & (sel < 0.08)] = np.float32(0.0)
        sub = (sel >= 0.08) & (sel < 0.12)
        X[sub] = (np.float32(1e-41) * np.where(sel[sub] < 0.10, 1, -1)).astype(np.float32)
        big = (sel >= 0.12) & (sel < 0.14)
        X[big] = (np.float32(3e30) * np.where(sel[big] < 0.13, 1, -1)).astype(np.float32)
        return X
    raise ValueError(dist)


def client_weights(kind: str, K: int, seed: int):
    """Python-level weights exactly as the reference's callers produce them.

    fedavg   int num_samples[train] ~ U{50..600}      (fedavg.py:181-191 -> utils.py:42-43)
    adabest  1                                        (adabest.py:158-166)
    fednova  float n / num_steps                      (fednova.py:58-59)
    bigint   ints around 2**25 (not all fp32-representable)
    """
    if kind == "fedavg":
        return [int(v) for v in randint(seed * 13 + 11, K, 50, 600)]
    if kind == "adabest":
        return [1] * K
    if kind == "fednova":
        n = randint(seed * 13 + 11, K, 50, 600)
        steps = randint(seed * 13 + 12, K, 1, 40)
        return [int(a) / int(b) for a, b in zip(n, steps)]
    if kind == "bigint":
        return [int(v) for v in randint(seed * 13 + 14, K, 2**25 - 50, 2**25 + 50)]
    raise ValueError(kind)


def client_messages(X: np.ndarray, weights, diverged_at=None, device=None):
    """Client messages shaped like FedAvg.send_to_server's return
    (fedsim/distributed/centralized/training/fedavg.py:173-179).  The train
    split's sample count carries the weight; per-split scalar metrics exercise
    serial_aggregation's metric path (training/utils.py:47-51)."""
    import torch

    msgs = []
    for k in range(X.shape[0]):
        w = weights[k]
        n = w if isinstance(w, int) else int(round(w * 10))
        params = torch.from_numpy(X[k].copy())
        if device is not None:
            params = params.to(device)
        msgs.append(
            dict(
                local_params=params,
                num_steps=max(1, n // 32),
                diverged=(diverged_at is not None and k == diverged_at),
                num_samples={"train": n, "test": 100 + k},
                metrics={"train": {"loss": 2.0 + 0.01 * k, "acc": 0.1 * (k % 7)},
                         "test": {"acc": 0.05 * (k % 5)}},
            )
        )
    return msgs


def cloud_vector(P: int, seed: int) -> np.ndarray:
    return (0.05 * gauss(seed * 7919 + 7, P) + 1e-2 * gauss(seed * 5 + 99991, P)).astype(
        np.float32
    )


def teacher_vectors(init: np.ndarray, K: int, seed: int, n_base: int = 16, scale: float = 0.02):
    """K FedDF teacher vectors around a model's init cloud, generated one at a
    time (nothing K x P is ever held): teacher k = fl32(init + fl32(c_k *
    roll(D_{k mod n_base}, 7919 k mod P))), with n_base shared deltas
    D_j = fl32(scale * N(0, 1)) and c_k in [0.5, 1.5).  Only fp32 elementwise
    multiplies and adds (one rounding each) and a permutation, so every
    platform regenerates the same bits; 16 hashed deltas keep 1000 teachers at
    a few seconds instead of a hash per teacher."""
    init = np.ascontiguousarray(init, dtype=np.float32)
    P = init.size
    D = [(scale * gauss(seed * 7919 + 31 + j, P)).astype(np.float32) for j in range(n_base)]
    c = (0.5 + uniform01(seed * 13 + 5, K)).astype(np.float32)
    for k in range(K):
        d = np.roll(D[k % n_base], (k * 7919) % P)
        yield init + c[k] * d


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
