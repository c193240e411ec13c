"""Typed Python wrappers over the libfedagg C-ABI (include/fedagg.h).

Each wrapper validates shapes / dtypes / devices / alignment on the host, then
launches on the current torch HIP stream.  None of them has a CPU fallback:
they raise if the tensors are not fp32 HIP tensors or if libfedagg is absent.

Reference arithmetic each op reproduces bit for bit:
  reduce      SerialAggregator.add   fedsim/utils/aggregators.py:17-40
              (+ FINALIZE: get/pop   fedsim/utils/aggregators.py:56-60,118-122)
  finalize    SerialAggregator.pop   fedsim/utils/aggregators.py:118-122
  finalize_f64  the same for fp64 sums (the dtype-generic keys)
  fedavg_sgd  FedAvg.optimize        fedsim/distributed/centralized/training/fedavg.py:199-203
  adabest_sgd AdaBest.optimize       fedsim/distributed/centralized/training/adabest.py:178-188
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native
from ._native import FEDAGG_FAST, FEDAGG_FINALIZE, FEDAGG_INIT, FEDAGG_NT, FEDAGG_SCALAR, check

__all__ = [
    "fl32",
    "reduce_slab",
    "reduce_rows",
    "finalize",
    "finalize_f64",
    "reduce_rows_ref",
    "fedavg_sgd",
    "adabest_sgd",
    "tuning_flags",
]


def fl32(x) -> float:
    """Round a Python int/float to the nearest fp32, as ATen does when a Python
    scalar meets an fp32 tensor (``value * weight``, ``v / w``)."""
    return float(np.float32(x))


def tuning_flags(unroll: int = 0, vpt: int = 0, nt: bool = False, bs: int = 0,
                 mapping: str = "auto", fast: bool = False) -> int:
    """Kernel tuning bits (include/fedagg.h): k-unroll, float4 slots per lane
    (row-major / pointer-table layouts), non-temporal loads, the workgroup
    size of the column-blocked layout, and the column mapping (``"auto"``, ``"wide"`` = f32x4
    slots, ``"narrow1"`` / ``"narrow2"`` / ``"narrow4"`` = one / two / four
    columns per lane).
    ``fast``: FEDAGG_FAST, the reordered split-K mode for small P (normwise
    parity, not bitwise).  0 / False / "auto" = library default."""
    sel = {0: 0, 4: 1, 8: 2, 16: 3, 2: 4, 32: 5}[unroll]
    msel = {"auto": 0, "wide": 1, "narrow1": 2, "narrow2": 3, "narrow4": 4}[mapping]
    vsel = {0: 0, 1: 1, 2: 2, 4: 3}[vpt]
    bsel = {0: 0, 256: 1, 512: 2, 1024: 3}[bs]
    return ((sel << _native.FEDAGG_UNROLL_SHIFT) | (vsel << _native.FEDAGG_VPT_SHIFT)
            | (bsel << _native.FEDAGG_BS_SHIFT) | (FEDAGG_NT if nt else 0)
            | (msel << _native.FEDAGG_MAP_SHIFT) | (_native.FEDAGG_FAST if fast else 0))


# Tuned defaults for the column-blocked reduce (profiles/r01_sweep*/: K=1000 at
# P=25M and P=1.09M on MI355X): non-temporal client-row loads, 256-lane
# workgroups; k-unroll 4 for C=4096, 2 for the narrower blocks.
DEFAULT_FLAGS = tuning_flags(unroll=4, nt=True)
_FLAGS_BY_C = {4096: tuning_flags(unroll=4, nt=True), 2048: tuning_flags(unroll=2, nt=True),
               1024: tuning_flags(unroll=2, nt=True)}
_MIN_WORKGROUPS = 2048  # ~8 per CU: below this, narrower column blocks win


def column_mapping(P: int, flags: int = 0, max_vw: int = 4, B: int = 1000):
    """The reduce kernel the library picks for B rows x P columns under ``flags``
    (fedagg_column_mapping): ``("wide", None)`` for the f32x4-slot kernels,
    else ``("narrow<vw>", unroll)``.  ``max_vw``: the most columns per lane
    the operands' alignment allows (P's divisibility is applied here)."""
    vw, u = ctypes.c_int(), ctypes.c_int()
    max_vw = min(max_vw, 4 if P % 4 == 0 else 2 if P % 2 == 0 else 1)
    check(_native.load().fedagg_column_mapping(P, B, flags, max_vw, ctypes.byref(vw),
                                                ctypes.byref(u)), "fedagg_column_mapping")
    return ("wide", None) if vw.value == 0 else (f"narrow{vw.value}", u.value)


_ROWS_KINDS = {1: "narrow1", 2: "narrow2", 3: "narrow4", 4: "wide", 5: "tile4x8",
               6: "tile8x4", 7: "splitk", 8: "flat"}


def rows_plan(P: int, B: int, flags: int = 0, aligned: bool = True) -> str:
    """The kernel fedagg_reduce_rows_f32 launches for B borrowed rows x P
    columns under ``flags`` (fedagg_rows_plan; host-side): ``"tile4x8"`` /
    ``"tile8x4"`` (the wide per-row tiles of the default flags), ``"narrow1"``
    / ``"narrow2"`` / ``"narrow4"`` / ``"wide"`` (the column kernels a tuning
    field names), ``"splitk"`` (FEDAGG_FAST) or ``"flat"``."""
    kind = ctypes.c_int()
    check(_native.load().fedagg_rows_plan(P, B, flags, 1 if aligned else 0, ctypes.byref(kind)),
          "fedagg_rows_plan")
    return _ROWS_KINDS[kind.value]


def choose_block_cols(P: int) -> int:
    """Widest column block that still yields >= ~8 workgroups per CU (the
    sweeps: C=4096 best at P=25M, C=1024 best at P=1.09M)."""
    for C in (4096, 2048):
        if (P + C - 1) // C >= _MIN_WORKGROUPS:
            return C
    return 1024


def default_flags(C: int) -> int:
    return _FLAGS_BY_C[C]


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_hip_f32(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must live on a HIP device, got {t.device}")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def reduce_slab(
    X: torch.Tensor,
    w32: torch.Tensor,
    out: torch.Tensor,
    acc_in: Optional[torch.Tensor] = None,
    W: Optional[float] = None,
    P: Optional[int] = None,
    flags: int = 0,
) -> torch.Tensor:
    """Weighted sequential reduction of the rows of ``X`` ([B, ldx] fp32, rows
    contiguous) into ``out`` ([P]).  ``acc_in=None`` starts from +0.0; ``W`` not
    None divides by fl32(W) on the way out (SerialAggregator.pop)."""
    _require_hip_f32(X, "X")
    _require_hip_f32(w32, "w32")
    _require_hip_f32(out, "out")
    if X.dim() != 2 or X.stride(1) != 1:
        raise ValueError("X must be 2-D with contiguous rows")
    B, ldx = X.shape[0], X.stride(0) if X.shape[0] > 1 else X.shape[1]
    if P is None:
        P = X.shape[1]
    if P > X.shape[1]:
        raise ValueError("P exceeds the row length of X")
    if w32.numel() < B or not w32.is_contiguous():
        raise ValueError("w32 must be contiguous with at least B entries")
    if out.numel() < P or not out.is_contiguous():
        raise ValueError("out must be contiguous with at least P entries")
    f = flags
    if acc_in is None:
        f |= FEDAGG_INIT
    else:
        _require_hip_f32(acc_in, "acc_in")
        if acc_in.numel() < P or not acc_in.is_contiguous():
            raise ValueError("acc_in must be contiguous with at least P entries")
    W32 = 0.0
    if W is not None:
        f |= FEDAGG_FINALIZE
        W32 = fl32(W)
    lib = _native.load()
    rc = lib.fedagg_reduce_f32(
        X.data_ptr(), ldx, w32.data_ptr(), B, P, _ptr(acc_in), out.data_ptr(),
        W32, f, _stream_ptr(out.device),
    )
    check(rc, "fedagg_reduce_f32")
    return out


def reduce_rows(
    rows: Sequence[torch.Tensor],
    w32: torch.Tensor,
    out: torch.Tensor,
    acc_in: Optional[torch.Tensor] = None,
    W: Optional[float] = None,
    flags: int = 0,
    table: Optional[torch.Tensor] = None,
    checked: bool = False,
) -> torch.Tensor:
    """Same as :func:`reduce_slab` but each client row is its own HIP tensor
    (no packing copy).  ``table`` may pass a pre-filled int64 device tensor of
    row pointers; otherwise one is built and uploaded.  ``checked``: every row
    is known to be a contiguous, 16-B aligned fp32 HIP tensor of P elements
    (skip the per-row checks)."""
    _require_hip_f32(out, "out")
    _require_hip_f32(w32, "w32")
    P = out.numel()
    B = len(rows)
    aligned = True
    for i, r in enumerate(() if checked else rows):
        _require_hip_f32(r, f"rows[{i}]")
        if r.numel() != P or not r.is_contiguous():
            raise ValueError(f"rows[{i}] must be contiguous with {P} elements")
        if r.data_ptr() % 16:
            aligned = False
    if table is None:
        table = row_table(rows, out.device)
    f = flags
    if acc_in is None:
        f |= FEDAGG_INIT
    else:
        _require_hip_f32(acc_in, "acc_in")
    W32 = 0.0
    if W is not None:
        f |= FEDAGG_FINALIZE
        W32 = fl32(W)
    lib = _native.load()
    if not aligned:
        f |= FEDAGG_SCALAR  # some row is not 16-B aligned: 4-byte-per-lane path
    rc = lib.fedagg_reduce_rows_f32(
        table.data_ptr(), w32.data_ptr(), B, P, _ptr(acc_in), out.data_ptr(), W32, f,
        _stream_ptr(out.device),
    )
    check(rc, "fedagg_reduce_rows_f32")
    return out


BLOCK_COLS = (1024, 2048, 4096)


def blocked_shape(K: int, P: int, C: int = 2048):
    """Shape [ceil(P/C), K, C] of a column-blocked slab (see fedagg.h)."""
    if C not in BLOCK_COLS:
        raise ValueError(f"C must be one of {BLOCK_COLS}")
    return ((P + C - 1) // C, K, C)


def to_blocked(X: torch.Tensor, C: int = 2048, kcap: Optional[int] = None) -> torch.Tensor:
    """Repack a [K, P] tensor into the column-blocked layout (copy), with
    ``kcap`` >= K rows of capacity per column block (rows K.. are zero)."""
    K, P = X.shape
    kcap = K if kcap is None else kcap
    nb, _, _ = blocked_shape(K, P, C)
    Xb = torch.zeros((nb, kcap, C), dtype=X.dtype, device=X.device)
    full = P // C
    if full:
        Xb[:full, :K].copy_(X[:, : full * C].reshape(K, full, C).transpose(0, 1))
    if P % C:
        Xb[full, :K, : P % C].copy_(X[:, full * C:])
    return Xb


def reduce_blocked(
    Xb: torch.Tensor,
    w32: torch.Tensor,
    out: torch.Tensor,
    B: Optional[int] = None,
    acc_in: Optional[torch.Tensor] = None,
    W: Optional[float] = None,
    flags: int = 0,
    r0: int = 0,
) -> torch.Tensor:
    """Reduce rows r0..r0+B-1 of a column-blocked slab ``Xb`` ([nblk, Kcap, C])."""
    _require_hip_f32(Xb, "Xb")
    _require_hip_f32(w32, "w32")
    _require_hip_f32(out, "out")
    if Xb.dim() != 3 or not Xb.is_contiguous():
        raise ValueError("Xb must be a contiguous [nblk, Kcap, C] tensor")
    nb, Kcap, C = Xb.shape
    P = out.numel()
    if nb != (P + C - 1) // C:
        raise ValueError("Xb block count does not match out's length")
    B = Kcap - r0 if B is None else B
    if w32.numel() < B:
        raise ValueError("w32 too short")
    if r0 < 0 or B < 0 or r0 + B > Kcap:
        raise ValueError("row range outside the slab")
    f = flags
    if acc_in is None:
        f |= FEDAGG_INIT
    else:
        _require_hip_f32(acc_in, "acc_in")
    W32 = 0.0
    if W is not None:
        f |= FEDAGG_FINALIZE
        W32 = fl32(W)
    rc = _native.load().fedagg_reduce_blocked_f32(
        Xb.data_ptr() + 4 * r0 * C, Kcap, C, w32.data_ptr(), B, P, _ptr(acc_in),
        out.data_ptr(), W32, f, _stream_ptr(out.device),
    )
    check(rc, "fedagg_reduce_blocked_f32")
    return out


def pack_row(src: torch.Tensor, Xb: torch.Tensor, r: int, stream=None) -> None:
    """Copy one client vector (contiguous fp32; pinned host or HIP memory) into
    row ``r`` of the column-blocked slab ``Xb``, ordered on ``stream``
    (default: the current stream of Xb's device): a copy kernel, reading a
    page-locked host vector in place over PCIe, or a 2-D DMA where the source
    is not 16-byte aligned.

    The copy is asynchronous and bypasses torch's copy bookkeeping: the caller
    keeps ``src`` alive and unmodified until ``stream`` has passed the copy
    (the aggregator's staging ring does this with per-slot events)."""
    _require_hip_f32(Xb, "Xb")
    if not isinstance(src, torch.Tensor) or src.dtype != torch.float32:
        raise TypeError("src must be a float32 tensor")
    if not src.is_contiguous():
        raise ValueError("src must be contiguous")
    if src.device.type == "cuda" and src.device != Xb.device:
        raise ValueError("device src must live on Xb's device")
    nb, Kcap, C = Xb.shape
    P = src.numel()
    if nb != (P + C - 1) // C or not 0 <= r < Kcap:
        raise ValueError("src / slab shape mismatch")
    s = stream.cuda_stream if stream is not None else _stream_ptr(Xb.device)
    rc = _native.load().fedagg_pack_row_f32(src.data_ptr(), P, Xb.data_ptr(), Kcap, C, r, s)
    check(rc, "fedagg_pack_row_f32")


def segments(tensors: Sequence[torch.Tensor], device: torch.device):
    """([[pointer, first column, length], ...], P): the segments that
    concatenate ``tensors`` (fedagg_pack_segments_f32).  Adjacent tensors that
    are adjacent in memory -- a model's parameters after
    ``vector_to_parameters`` made them views of one vector -- are one segment.
    Every tensor must be a contiguous fp32 tensor on ``device``."""
    segs = []
    P = 0
    for i, t in enumerate(tensors):
        if t.dtype != torch.float32 or t.device != device or not t.is_contiguous():
            raise ValueError(f"tensors[{i}] must be a contiguous float32 tensor on {device}")
        n = t.numel()
        if n == 0:
            continue
        ptr = t.data_ptr()
        if segs and segs[-1][0] + 4 * segs[-1][2] == ptr:
            segs[-1][2] += n
        else:
            segs.append([ptr, P, n])
        P += n
    return segs, P


_TABLES: dict = {}  # (device, segments) -> device table; a model's layout repeats


def segment_table(tensors: Sequence[torch.Tensor], device: torch.device):
    """(device int64 table, number of segments, P) for fedagg_pack_segments_f32."""
    segs, P = segments(tensors, device)
    key = (device, tuple(v for seg in segs for v in seg))
    table = _TABLES.get(key)
    if table is None:
        if len(_TABLES) > 64:
            _TABLES.clear()
        host = torch.tensor(list(key[1]) or [0, 0, 0], dtype=torch.int64, pin_memory=True)
        table = _TABLES[key] = host.to(device, non_blocking=True)
    return table, len(segs), P


def pack_segments(tensors: Sequence[torch.Tensor], Xb: torch.Tensor, r: int) -> int:
    """Write the concatenation of ``tensors`` (a model's parameters, in order)
    into row ``r`` of the column-blocked slab ``Xb`` in one launch:
    vectorize_module straight into the slab.  One segment (parameters that are
    views of one vector, as a round's client models are) is the plain row
    pack (fedagg_pack_row_f32); several go through a device table of segments
    (fedagg_pack_segments_f32, tables cached per layout).  Returns P."""
    _require_hip_f32(Xb, "Xb")
    nb, Kcap, C = Xb.shape
    segs, P = segments(tensors, Xb.device)
    if nb != (P + C - 1) // C or not 0 <= r < Kcap:
        raise ValueError("tensors / slab shape mismatch")
    lib = _native.load()
    if len(segs) == 1 and segs[0][0] % 16 == 0:
        rc = lib.fedagg_pack_row_f32(segs[0][0], P, Xb.data_ptr(), Kcap, C, r,
                                     _stream_ptr(Xb.device))
        check(rc, "fedagg_pack_row_f32")
        return P
    table, nseg, _ = segment_table(tensors, Xb.device)
    rc = lib.fedagg_pack_segments_f32(table.data_ptr(), nseg, P, Xb.data_ptr(), Kcap, C, r,
                                      _stream_ptr(Xb.device))
    check(rc, "fedagg_pack_segments_f32")
    return P


def unpack_row(Xb: torch.Tensor, r: int, P: int, out: Optional[torch.Tensor] = None):
    """Row ``r`` of a column-blocked slab as a contiguous [P] vector
    (fedagg_unpack_row_f32)."""
    _require_hip_f32(Xb, "Xb")
    nb, Kcap, C = Xb.shape
    if nb != (P + C - 1) // C or not 0 <= r < Kcap:
        raise ValueError("slab / row mismatch")
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=Xb.device)
    _require_hip_f32(out, "out")
    if out.numel() != P or not out.is_contiguous() or out.device != Xb.device:
        raise ValueError(f"out must be a contiguous [{P}] tensor on {Xb.device}")
    rc = _native.load().fedagg_unpack_row_f32(Xb.data_ptr(), Kcap, C, r, P, out.data_ptr(),
                                              _stream_ptr(Xb.device))
    check(rc, "fedagg_unpack_row_f32")
    return out


def _rows_contiguous(slab: torch.Tensor) -> bool:
    """[K, P] with unit column stride and a row pitch >= P (a slab whose rows
    are padded to 16 B, as TeacherEnsemble allocates it)."""
    return slab.stride(1) == 1 and (slab.shape[0] <= 1 or slab.stride(0) >= slab.shape[1])


def _row_pitch(slab: torch.Tensor) -> int:
    return slab.stride(0) if slab.shape[0] > 1 else slab.shape[1]


def teacher_linear(x: torch.Tensor, slab: torch.Tensor, w_off: int, b_off: int, in_f: int,
                   out_f: int, shared: bool, relu: bool = False) -> torch.Tensor:
    """One nn.Linear layer of the K teacher models whose flat parameter
    vectors are the rows of ``slab`` ([K, P], parameters_to_vector layout),
    on the matrix cores (fedagg_teacher_linear_f32).  ``x``: [M, in] shared by
    every teacher (``shared``) or [K, M, in].  Returns y [K, M, out]
    (ReLU applied when ``relu``).  b_off = -1: no bias."""
    _require_hip_f32(x, "x")
    _require_hip_f32(slab, "slab")
    if slab.dim() != 2 or not _rows_contiguous(slab) or x.device != slab.device:
        raise ValueError("slab must be a [K, P] tensor with contiguous rows on x's device")
    if not x.is_contiguous() or x.shape[-1] != in_f:
        raise ValueError(f"x must be contiguous with a last dimension of {in_f}")
    K, P = slab.shape
    if w_off < 0 or w_off + in_f * out_f > P or (b_off >= 0 and b_off + out_f > P):
        raise ValueError("layer offsets outside the parameter vector")
    M = x.numel() // in_f if shared else x.numel() // (in_f * max(K, 1))
    if not shared and x.shape[0] != K:
        raise ValueError("a per-teacher x must have K rows in its first dimension")
    y = torch.empty((K, M, out_f), dtype=torch.float32, device=x.device)
    rc = _native.load().fedagg_teacher_linear_f32(
        x.data_ptr(), 0 if shared else M * in_f, slab.data_ptr(), _row_pitch(slab), w_off, b_off,
        K, M, in_f, out_f, y.data_ptr(), _native.FEDAGG_RELU if relu else 0, _stream_ptr(x.device))
    check(rc, "fedagg_teacher_linear_f32")
    return y


def conv_shape(x_shape, out_channels: int, kernel_size, stride, padding) -> "_native.Conv2dShape":
    """struct fedagg_conv2d_shape of a conv over x [..., M, C, H, W] with
    ``padding`` = (top, bottom, left, right)."""
    M, C, H, W = x_shape[-4:]
    KH, KW = kernel_size
    sh, sw = stride
    pt, pb, pl, pr = padding
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    return _native.Conv2dShape(M, C, H, W, out_channels, KH, KW, sh, sw, pt, pl, OH, OW)


def conv_order(x_shape, out_channels: int, kernel_size, stride, padding,
               gather: bool = False) -> int:
    """The fmaf chain order teacher_conv2d takes for this geometry
    (fedagg_conv_order): 0 = (c, kh, kw), else the LDS kernel's channel chunk."""
    s = conv_shape(x_shape, out_channels, kernel_size, stride, padding)
    return int(_native.load().fedagg_conv_order(ctypes.byref(s),
                                                _native.FEDAGG_CONV_GATHER if gather else 0))


def _pool_flags(pool) -> int:
    """Conv flags fusing ``pool`` = (kh, kw, sh, sw, ph, pw), or -1 when it is
    not the 2 x 2 / stride 2 pool (padding 0 or 1) the conv kernel fuses."""
    if pool is None:
        return 0
    kh, kw, sh, sw, ph, pw = pool
    if (kh, kw, sh, sw) != (2, 2, 2, 2) or ph != pw or ph not in (0, 1):
        return -1
    return _native.FEDAGG_CONV_MAXPOOL2 | (_native.FEDAGG_CONV_POOL_PAD1 if ph else 0)


def conv_pool_fusable(x_shape, out_channels: int, kernel_size, stride, padding, pool) -> bool:
    """Whether teacher_conv2d(..., pool=pool) fuses the max pool into the conv
    (fedagg_conv_pool_fusable: the LDS-resident kernel for 1 or 3 input
    channels; SimpleCNN's conv1 -> relu -> max_pool2d(2, 2, padding=1))."""
    f = _pool_flags(pool)
    if f <= 0:
        return False
    s = conv_shape(x_shape, out_channels, kernel_size, stride, padding)
    return bool(_native.load().fedagg_conv_pool_fusable(ctypes.byref(s), f))


def teacher_conv2d(x: torch.Tensor, slab: torch.Tensor, w_off: int, b_off: int,
                   out_channels: int, kernel_size, stride, padding, shared: bool,
                   relu: bool = False, gather: bool = False, pool=None) -> torch.Tensor:
    """One nn.Conv2d (groups 1, dilation 1, zero padding) of the K teachers
    whose flat parameter vectors are the rows of ``slab`` ([K, P]), as an
    implicit GEMM on the matrix cores (fedagg_teacher_conv2d_f32).  ``x``:
    [M, C, H, W] shared by every teacher (``shared``) or [K, M, C, H, W].
    ``padding`` = (top, bottom, left, right) zeros.  Returns
    y [K, M, OC, OH, OW] (ReLU applied when ``relu``).  b_off = -1: no bias.
    ``gather``: the im2col-gather kernel even where the LDS one applies.
    ``pool`` = (2, 2, 2, 2, p, p), p in {0, 1}: the max pool after the layer
    fused into its store (conv_pool_fusable must hold); y is then the pooled
    [K, M, OC, PH, PW], the same bits as pad_lrn_maxpool(y, pool=pool)."""
    _require_hip_f32(x, "x")
    _require_hip_f32(slab, "slab")
    if slab.dim() != 2 or not _rows_contiguous(slab) or x.device != slab.device:
        raise ValueError("slab must be a [K, P] tensor with contiguous rows on x's device")
    K, P = slab.shape
    if not x.is_contiguous() or x.dim() != (4 if shared else 5):
        raise ValueError("x must be a contiguous [M, C, H, W] (shared) or [K, M, C, H, W] tensor")
    if not shared and x.shape[0] != K:
        raise ValueError("a per-teacher x must have K rows in its first dimension")
    M, C, H, W = x.shape[-4:]
    KH, KW = kernel_size
    sh, sw = stride
    pt, pb, pl, pr = padding
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    if OH <= 0 or OW <= 0:
        raise ValueError("the padded input is smaller than the kernel")
    R = C * KH * KW
    if w_off < 0 or w_off + out_channels * R > P or (b_off >= 0 and b_off + out_channels > P):
        raise ValueError("layer offsets outside the parameter vector")
    pflags = _pool_flags(pool)
    if pflags < 0:
        raise ValueError(f"pool {pool} is not a 2 x 2 / stride 2 max pool with padding 0 or 1")
    shape = _native.Conv2dShape(M, C, H, W, out_channels, KH, KW, sh, sw, pt, pl, OH, OW)
    flags = ((_native.FEDAGG_RELU if relu else 0) | (_native.FEDAGG_CONV_GATHER if gather else 0)
             | pflags)
    if pflags:
        if not _native.load().fedagg_conv_pool_fusable(ctypes.byref(shape), flags):
            raise ValueError("the conv kernel does not fuse this pool for this shape")
        ph = pool[4]
        OH, OW = (OH + 2 * ph - 2) // 2 + 1, (OW + 2 * ph - 2) // 2 + 1
    y = torch.empty((K, M, out_channels, OH, OW), dtype=torch.float32, device=x.device)
    rc = _native.load().fedagg_teacher_conv2d_f32(
        x.data_ptr(), 0 if shared else M * C * H * W, slab.data_ptr(), _row_pitch(slab), w_off,
        b_off, K, ctypes.byref(shape), y.data_ptr(), flags, _stream_ptr(x.device))
    check(rc, "fedagg_teacher_conv2d_f32")
    return y


def pool_args(shape, pads=(0, 0, 0, 0), lrn=None, pool=None,
              planes: bool = False) -> "_native.PoolArgs":
    """struct fedagg_pool_args for an input of ``shape`` (..., C, H, W):
    ``pads`` (top, bottom, left, right) zeros, ``lrn`` (size, alpha, beta, k)
    or None, ``pool`` (kh, kw, sh, sw, ph, pw) or None.  ``planes``: take the
    per-block kernels instead of the sliding channel window
    (FEDAGG_POOL_PLANES; same bits, A/B and tests)."""
    C, H, W = shape[-3:]
    N = 1
    for d in shape[:-3]:
        N *= int(d)
    size, alpha, beta, k = lrn if lrn is not None else (0, 0.0, 0.0, 0.0)
    pk = pool if pool is not None else (0, 0, 0, 0, 0, 0)
    top, bottom, left, right = pads
    return _native.PoolArgs(
        N=N, C=C, H=H, W=W, pad_top=top, pad_bottom=bottom, pad_left=left, pad_right=right,
        lrn_size=size, lrn_alpha=alpha, lrn_beta=beta, lrn_k=k,
        flags=_native.FEDAGG_POOL_PLANES if planes else 0,
        pool_kh=pk[0], pool_kw=pk[1], pool_sh=pk[2], pool_sw=pk[3], pool_ph=pk[4], pool_pw=pk[5])


def pool_output(args) -> tuple:
    """(OH, OW) of fedagg_pad_lrn_maxpool_f32, or raise ValueError when the
    library rejects the chain's shape (the caller keeps torch for it)."""
    oh, ow, cb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = _native.load().fedagg_pool_output(ctypes.byref(args), ctypes.byref(oh), ctypes.byref(ow),
                                           ctypes.byref(cb))
    if rc != 0:
        raise ValueError("pad / local_response_norm / max_pool2d chain not supported")
    return oh.value, ow.value


def pad_lrn_maxpool(x: torch.Tensor, pads=(0, 0, 0, 0), lrn=None, pool=None,
                    planes: bool = False) -> torch.Tensor:
    """F.pad (zeros) -> F.local_response_norm -> F.max_pool2d over the last
    three dimensions (C, H, W) of ``x`` in one pass
    (fedagg_pad_lrn_maxpool_f32); leading dimensions are images."""
    _require_hip_f32(x, "x")
    if not x.is_contiguous() or x.dim() < 3:
        raise ValueError("x must be a contiguous (..., C, H, W) tensor")
    args = pool_args(x.shape, pads, lrn, pool, planes=planes)
    OH, OW = pool_output(args)
    y = torch.empty((*x.shape[:-2], OH, OW), dtype=torch.float32, device=x.device)
    rc = _native.load().fedagg_pad_lrn_maxpool_f32(x.data_ptr(), ctypes.byref(args), y.data_ptr(),
                                                   _stream_ptr(x.device))
    check(rc, "fedagg_pad_lrn_maxpool_f32")
    return y


def finalize(acc: torch.Tensor, W, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = fl32(acc / fl32(W)) — SerialAggregator.pop's true division."""
    _require_hip_f32(acc, "acc")
    if out is None:
        out = torch.empty_like(acc)
    _require_hip_f32(out, "out")
    rc = _native.load().fedagg_finalize_f32(
        acc.data_ptr(), fl32(W), acc.numel(), out.data_ptr(), _stream_ptr(acc.device)
    )
    check(rc, "fedagg_finalize_f32")
    return out


def finalize_f64(acc: torch.Tensor, W, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = acc / float(W) in f64 (IEEE true division) — SerialAggregator.pop's
    ``v / w`` for an fp64 sum (fedagg_finalize_f64)."""
    if not isinstance(acc, torch.Tensor) or acc.dtype != torch.float64:
        raise TypeError("acc must be a float64 torch.Tensor")
    if acc.device.type != "cuda":
        raise ValueError(f"acc must live on a HIP device, got {acc.device}")
    if out is None:
        out = torch.empty_like(acc, memory_format=torch.contiguous_format)
    if out.dtype != torch.float64 or out.device != acc.device or out.numel() != acc.numel():
        raise ValueError("out must be a float64 tensor of acc's size on acc's device")
    rc = _native.load().fedagg_finalize_f64(
        acc.data_ptr(), float(W), acc.numel(), out.data_ptr(), _stream_ptr(acc.device)
    )
    check(rc, "fedagg_finalize_f64")
    return out


_REF_DTYPES = {torch.bfloat16: (_native.FEDAGG_DTYPE_BF16, torch.float32),
               torch.float16: (_native.FEDAGG_DTYPE_F16, torch.float32),
               torch.float64: (_native.FEDAGG_DTYPE_F64, torch.float64)}


def reduce_rows_ref(rows: Sequence[torch.Tensor], weights: Sequence, out: torch.Tensor,
                    acc_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The reference's ``add`` arithmetic over bf16 / fp16 / fp64 rows
    (fedagg_reduce_rows_ref): ``out = acc_in + x_0 * w_0 + ...`` rounded per
    product and per sum in the rows' dtype, in order; ``acc_in=None``: from
    the reference's ``0 + first product``.  ``weights`` are the Python
    weights (fl32 for bf16 / fp16, as ATen's opmath takes them)."""
    if out.dtype not in _REF_DTYPES:
        raise TypeError(f"reduce_rows_ref takes bf16 / fp16 / fp64 tensors, got {out.dtype}")
    code, wdt = _REF_DTYPES[out.dtype]
    dev = out.device
    if dev.type != "cuda" or not out.is_contiguous():
        raise ValueError("out must be a contiguous HIP tensor")
    P, B = out.numel(), len(rows)
    if len(weights) != B:
        raise ValueError("one weight per row")
    aligned = out.data_ptr() % 16 == 0
    for i, r in enumerate(rows):
        if r.dtype != out.dtype or r.device != dev or r.numel() != P or not r.is_contiguous():
            raise ValueError(f"rows[{i}] must be a contiguous {out.dtype} tensor of {P} "
                             f"elements on {dev}")
        aligned = aligned and r.data_ptr() % 16 == 0
    if acc_in is not None:
        if acc_in.dtype != out.dtype or acc_in.device != dev or acc_in.numel() != P or \
                not acc_in.is_contiguous():
            raise ValueError("acc_in must match out")
        aligned = aligned and acc_in.data_ptr() % 16 == 0
    elif B == 0:
        raise ValueError("no rows and no acc_in")
    table = row_table_from_ptrs([r.data_ptr() for r in rows], dev) if B else None
    wv = torch.tensor([fl32(w) if wdt == torch.float32 else float(w) for w in weights],
                      dtype=wdt, pin_memory=True).to(dev, non_blocking=True) if B else None
    flags = (FEDAGG_INIT if acc_in is None else 0) | (0 if aligned else FEDAGG_SCALAR)
    rc = _native.load().fedagg_reduce_rows_ref(code, _ptr(table), _ptr(wv), B, P, _ptr(acc_in),
                                               out.data_ptr(), flags, _stream_ptr(dev))
    check(rc, "fedagg_reduce_rows_ref")
    return out


def fedavg_sgd(avg: torch.Tensor, cloud: torch.Tensor, lr: float,
               grad_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In-place FedAvg server step with plain SGD on ``cloud``."""
    _require_hip_f32(avg, "avg")
    _require_hip_f32(cloud, "cloud")
    if avg.numel() != cloud.numel():
        raise ValueError("avg / cloud size mismatch")
    if grad_out is not None:
        _require_hip_f32(grad_out, "grad_out")
    rc = _native.load().fedagg_fedavg_sgd_f32(
        avg.data_ptr(), fl32(lr), cloud.data_ptr(), _ptr(grad_out), cloud.numel(),
        _stream_ptr(cloud.device),
    )
    check(rc, "fedagg_fedavg_sgd_f32")
    return cloud


def feddyn_sgd(avg: torch.Tensor, cloud: torch.Tensor, h: torch.Tensor, ratio: float,
               lr: float, avg_prev: Optional[torch.Tensor] = None,
               grad_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In-place FedDyn server step (plain SGD): h += ratio*(cloud-avg); cloud
    steps toward avg - h; ``avg_prev`` <- avg.  ``ratio`` is the Python float
    weight / num_clients (rounded to fp32 here, as ATen does)."""
    for t, n in ((avg, "avg"), (cloud, "cloud"), (h, "h")):
        _require_hip_f32(t, n)
        if t.numel() != cloud.numel():
            raise ValueError(f"{n} size mismatch")
    for t, n in ((avg_prev, "avg_prev"), (grad_out, "grad_out")):
        if t is not None:
            _require_hip_f32(t, n)
    rc = _native.load().fedagg_feddyn_sgd_f32(
        avg.data_ptr(), fl32(ratio), fl32(lr), cloud.data_ptr(), h.data_ptr(), _ptr(avg_prev),
        _ptr(grad_out), cloud.numel(), _stream_ptr(cloud.device),
    )
    check(rc, "fedagg_feddyn_sgd_f32")
    return cloud


def host_mapped(t: torch.Tensor) -> bool:
    """Whether ``t`` is page-locked host memory the GPU reaches at its own
    address (fedagg_host_mapped: torch's pin_memory on this platform), so a
    kernel can read and write it in place over PCIe.  hipHostMalloc maps
    such memory into the address space of every GPU in the system
    (hip_runtime_api.h), so this holds for whichever device a kernel runs on
    (torch's host allocator shares its blocks across devices)."""
    if not isinstance(t, torch.Tensor) or t.device.type != "cpu" or not t.is_pinned():
        return False
    nbytes = t.numel() * t.element_size()
    return nbytes == 0 or _native.load().fedagg_host_mapped(t.data_ptr(), nbytes) == 1


def _require_hip_step(step: "ServerStep") -> None:
    """A kernel is launched on the step: it runs on a HIP device (its
    operands there or host-mapped, checked at construction)."""
    if step.device.type != "cuda":
        raise ValueError(f"cloud must live on a HIP device, got {step.device}")


ALGO = {"fedavg": _native.FEDAGG_ALGO_FEDAVG, "adabest": _native.FEDAGG_ALGO_ADABEST,
        "feddyn": _native.FEDAGG_ALGO_FEDDYN}


class ServerStep(object):
    """The operands of one server step (include/fedagg.h fedagg_step_args):
    the algorithm's pseudo-gradient + the full torch.optim.SGD update, in place
    on ``cloud`` (and ``aux`` / ``momentum_buf`` / ``avg_prev``).  Python
    scalars are rounded to fp32 exactly as ATen rounds them (fl32(-lr),
    fl32(1-damp)).

    ``apply(avg)`` runs it on a stored average (fedagg_server_step_f32);
    ``reduce_blocked_step(..., step)`` runs it fused into the last drain of a
    round, so the average never round-trips through HBM."""

    def __init__(self, algo: str, cloud: torch.Tensor, *, lr: float, momentum: float = 0.0,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                 maximize: bool = False, coef: float = 0.0,
                 aux: Optional[torch.Tensor] = None, avg_prev: Optional[torch.Tensor] = None,
                 momentum_buf: Optional[torch.Tensor] = None, momentum_init: bool = False,
                 grad_out: Optional[torch.Tensor] = None,
                 avg_out: Optional[torch.Tensor] = None,
                 device: Optional[torch.device] = None) -> None:
        if algo not in ALGO:
            raise ValueError(f"unknown algo {algo!r}")
        self.P = P = cloud.numel()
        self.cloud = cloud
        # the GPU the step runs on: every operand lives there, or is
        # page-locked host memory the kernel reads and writes in place over
        # PCIe (host_mapped: FedSim's device="cpu" server state)
        self.device = cloud.device if device is None else torch.device(device)
        operands = ((cloud, "cloud"), (aux, "aux"), (avg_prev, "avg_prev"),
                    (momentum_buf, "momentum_buf"), (grad_out, "grad_out"), (avg_out, "avg_out"))
        for t, n in operands:
            if t is not None:
                # the HIP-device check is made where a kernel is launched on
                # the operands (apply / reduce_*_step): a ServerStep is also
                # the description a sharded aggregator narrows per rank
                if not isinstance(t, torch.Tensor) or t.dtype != torch.float32:
                    raise TypeError(f"{n} must be a float32 tensor")
                if t.numel() != P or not t.is_contiguous():
                    raise ValueError(f"{n} must be contiguous with {P} elements")
                if t.device != self.device and not (
                        self.device.type == "cuda" and host_mapped(t)):
                    raise ValueError(f"{n} is on {t.device}, the step runs on {self.device}")
        self.algo = algo
        self.operands = {n: t for t, n in operands if t is not None}
        self._scalars = dict(lr=lr, momentum=momentum, dampening=dampening,
                             weight_decay=weight_decay, nesterov=nesterov, maximize=maximize,
                             coef=coef, momentum_init=momentum_init)
        self._keep = [t for t, _ in operands if t is not None]  # alive until launched
        self.sgd = _native.SgdParams(fl32(-lr), fl32(momentum), fl32(1 - dampening),
                                     fl32(weight_decay), int(bool(nesterov)),
                                     int(bool(maximize)))
        self.args = _native.StepArgs(ALGO[algo], fl32(coef), cloud.data_ptr(), _ptr(aux),
                                     _ptr(avg_prev), _ptr(momentum_buf),
                                     int(bool(momentum_init)), _ptr(grad_out), _ptr(avg_out),
                                     self.sgd)

    def aligned(self) -> bool:
        """Every operand 16-B aligned (required by the fused entry)."""
        return all(t.data_ptr() % 16 == 0 for t in self._keep)

    def narrow(self, lo: int, hi: int) -> "ServerStep":
        """The same step restricted to parameters [lo, hi) (views of every
        operand): what one rank of a parameter-sharded round runs."""
        views = {n: t[lo:hi] for n, t in self.operands.items()}
        cloud = views.pop("cloud")
        return ServerStep(self.algo, cloud, **self._scalars, **views, device=self.device)

    def outputs(self):
        """The operands the step writes (cloud and whichever of aux /
        avg_prev / momentum_buf / grad_out / avg_out it was given)."""
        return [t for n, t in self.operands.items()]

    def apply(self, avg: torch.Tensor) -> torch.Tensor:
        _require_hip_f32(avg, "avg")
        _require_hip_step(self)
        if avg.numel() != self.P or not avg.is_contiguous():
            raise ValueError(f"avg must be contiguous with {self.P} elements")
        if avg.device != self.device:
            raise ValueError(f"avg is on {avg.device}, the step runs on {self.device}")
        a = self.args
        rc = _native.load().fedagg_server_step_f32(
            a.algo, avg.data_ptr(), a.coef, a.cloud, a.aux, a.avg_prev, a.momentum_buf,
            a.momentum_init, a.grad_out, ctypes.byref(self.sgd), self.P,
            _stream_ptr(self.device),
        )
        check(rc, "fedagg_server_step_f32")
        avg_out = self.operands.get("avg_out")
        if avg_out is not None and avg_out.data_ptr() != avg.data_ptr():
            # the stored-average kernel has no avg_out operand: the fused
            # entries write it in their epilogue, this path copies it
            avg_out.copy_(avg)
        return self.cloud


def server_step(algo: str, avg: torch.Tensor, cloud: torch.Tensor, **kw) -> torch.Tensor:
    """ServerStep(algo, cloud, **kw).apply(avg)  (fedagg_server_step_f32)."""
    return ServerStep(algo, cloud, **kw).apply(avg)


def can_fuse_step(Xb: torch.Tensor, step: ServerStep) -> bool:
    """Whether fedagg_reduce_step_blocked_f32 accepts this slab and step."""
    return (Xb.dim() == 3 and Xb.shape[2] in BLOCK_COLS
            and Xb.shape[1] * Xb.shape[2] * 4 < (1 << 32) and step.aligned()
            and Xb.device == step.device)


# Below 2^24 columns the narrow kernels' grid is a few generations of resident
# waves, and a wave that carries the server step ends with a dependent load of
# the step's operands (cloud / aux) that keeps its slot idle: with B >= 128
# rows the separate epilogue launch is 1-7 % faster than the fused one there
# (profiles/r01bq/, r01br/, r01bs/; slab and borrowed rows, FedAvg and
# AdaBest), in spite of the 8 P bytes of the stored average.  Fewer rows pay
# more for the extra launch than the epilogue costs; from 2^24 columns on the
# two measure within noise and the fused pass saves the 8 P bytes.
_SPLIT_STEP_MIN_P = 1 << 20
_SPLIT_STEP_MAX_P = 1 << 24
_SPLIT_STEP_MIN_B = 128


def fuse_step_pays(P: int, B: int, borrowed: bool = False) -> bool:
    """Whether the last drain of a round should run the server step fused
    (fedagg_reduce_step_*_f32) rather than store the average and run
    fedagg_server_step_f32 after it.  Same results either way (bitwise).
    ``borrowed``: the rows are the caller's own tensors (pointer table); there
    the split pass stays ahead at every P from 2^20 on, +1.2-1.8 % at 25 M
    (profiles/r01cf/)."""
    if B < _SPLIT_STEP_MIN_B or P < _SPLIT_STEP_MIN_P:
        return True
    return not (borrowed or P < _SPLIT_STEP_MAX_P)


def reduce_blocked_step(
    Xb: torch.Tensor,
    w32: torch.Tensor,
    step: ServerStep,
    B: Optional[int] = None,
    acc_in: Optional[torch.Tensor] = None,
    W: Optional[float] = None,
    r0: int = 0,
    mapping: str = "auto",
    unroll: int = 0,
    flags: int = 0,
) -> torch.Tensor:
    """reduce_blocked(..., out=avg) then step.apply(avg), fused into one pass
    (fedagg_reduce_step_blocked_f32).  Returns step.cloud.  ``mapping`` as in
    :func:`tuning_flags` (same results); ``flags``: further tuning bits
    (e.g. FEDAGG_FAST) OR'ed in."""
    _require_hip_f32(Xb, "Xb")
    _require_hip_f32(w32, "w32")
    if Xb.dim() != 3 or not Xb.is_contiguous():
        raise ValueError("Xb must be a contiguous [nblk, Kcap, C] tensor")
    _require_hip_step(step)
    if step.device != Xb.device:
        raise ValueError(f"the step runs on {step.device}, the slab is on {Xb.device}")
    nb, Kcap, C = Xb.shape
    P = step.P
    if nb != (P + C - 1) // C:
        raise ValueError("Xb block count does not match the step's length")
    B = Kcap - r0 if B is None else B
    if w32.numel() < B:
        raise ValueError("w32 too short")
    if r0 < 0 or B < 0 or r0 + B > Kcap:
        raise ValueError("row range outside the slab")
    f = tuning_flags(unroll=unroll, mapping=mapping) | flags
    if acc_in is None:
        f |= FEDAGG_INIT
    else:
        _require_hip_f32(acc_in, "acc_in")
        if acc_in.numel() != P:
            raise ValueError("acc_in size mismatch")
    W32 = 0.0
    if W is not None:
        f |= FEDAGG_FINALIZE
        W32 = fl32(W)
    rc = _native.load().fedagg_reduce_step_blocked_f32(
        Xb.data_ptr() + 4 * r0 * C, Kcap, C, w32.data_ptr(), B, P, _ptr(acc_in), W32, f,
        ctypes.byref(step.args), _stream_ptr(Xb.device),
    )
    check(rc, "fedagg_reduce_step_blocked_f32")
    return step.cloud


def row_table(rows: Sequence[torch.Tensor], device: torch.device) -> torch.Tensor:
    """Device int64 table of the rows' data pointers (one pinned H2D copy,
    stream-ordered on the current stream)."""
    return row_table_from_ptrs([r.data_ptr() for r in rows], device)


def row_table_from_ptrs(ptrs: Sequence[int], device: torch.device) -> torch.Tensor:
    """row_table of pointers collected beforehand (as rows arrive)."""
    host = torch.tensor(list(ptrs) or [0], dtype=torch.int64, pin_memory=True)
    return host.to(device, non_blocking=True)


def reduce_rows_step(
    rows: Sequence[torch.Tensor],
    w32: torch.Tensor,
    step: ServerStep,
    acc_in: Optional[torch.Tensor] = None,
    W: Optional[float] = None,
    nt: bool = True,
    table: Optional[torch.Tensor] = None,
    mapping: str = "auto",
    unroll: int = 0,
    checked: bool = False,
    flags: int = 0,
) -> torch.Tensor:
    """reduce_rows(rows, ..., out=avg) then step.apply(avg), fused into one
    pass over the caller's own client tensors (fedagg_reduce_step_rows_f32):
    the zero-copy round of HBM-resident client vectors.  Returns step.cloud.
    ``checked``: the caller has already
    validated every row (the aggregator does at ``add``), skip the per-row
    checks."""
    _require_hip_f32(w32, "w32")
    _require_hip_step(step)
    P, dev = step.P, step.device
    B = len(rows)
    for i, r in enumerate(() if checked else rows):
        _require_hip_f32(r, f"rows[{i}]")
        if r.numel() != P or not r.is_contiguous() or r.data_ptr() % 16:
            raise ValueError(f"rows[{i}] must be contiguous, 16-B aligned, {P} elements")
        if r.device != dev:
            raise ValueError(f"rows[{i}] is on {r.device}, the step runs on {dev}")
    if w32.numel() < B:
        raise ValueError("w32 too short")
    if not step.aligned():
        raise ValueError("every server-step operand must be 16-B aligned")
    f = (FEDAGG_NT if nt else 0) | tuning_flags(mapping=mapping, unroll=unroll) | flags
    if acc_in is None:
        f |= FEDAGG_INIT
    else:
        _require_hip_f32(acc_in, "acc_in")
        if acc_in.numel() != P:
            raise ValueError("acc_in size mismatch")
    W32 = 0.0
    if W is not None:
        f |= FEDAGG_FINALIZE
        W32 = fl32(W)
    if table is None:
        table = row_table(rows, dev)
    rc = _native.load().fedagg_reduce_step_rows_f32(
        table.data_ptr(), w32.data_ptr(), B, P, _ptr(acc_in), W32, f,
        ctypes.byref(step.args), _stream_ptr(dev),
    )
    check(rc, "fedagg_reduce_step_rows_f32")
    return step.cloud


def adabest_sgd(avg: torch.Tensor, cloud: torch.Tensor, avg_prev: torch.Tensor,
                beta: float, lr: float,
                grad_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In-place AdaBest server step (plain SGD) on ``cloud``; ``avg_prev`` <- avg."""
    for t, n in ((avg, "avg"), (cloud, "cloud"), (avg_prev, "avg_prev")):
        _require_hip_f32(t, n)
        if t.numel() != cloud.numel():
            raise ValueError(f"{n} size mismatch")
    if grad_out is not None:
        _require_hip_f32(grad_out, "grad_out")
    rc = _native.load().fedagg_adabest_sgd_f32(
        avg.data_ptr(), fl32(beta), fl32(lr), cloud.data_ptr(), avg_prev.data_ptr(),
        _ptr(grad_out), cloud.numel(), _stream_ptr(cloud.device),
    )
    check(rc, "fedagg_adabest_sgd_f32")
    return cloud
