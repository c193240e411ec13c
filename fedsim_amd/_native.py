"""Loader for libfedagg.so, the HIP (gfx950) C-ABI declared in include/fedagg.h.

The library is linked against ``libamdhip64.so.7``.  PyTorch-ROCm ships its own
HIP runtime with the same soname, so torch MUST be imported first: the dynamic
linker then resolves our NEEDED entry to torch's already-loaded runtime and the
device pointers / hipStream_t handles torch hands us are valid in our calls.
Loading the library before torch would map a second HIP runtime; we check for
that and refuse.

There is deliberately no fallback: if the library is missing or cannot be
loaded, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

_LIB_NAME = "libfedagg.so"
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FEDAGG_LIB", os.path.join(_HERE, _LIB_NAME))

# Must match include/fedagg.h
ABI_VERSION = 6  # 2: round-2 entry points (teacher / pool / pack_segments / unpack_row);
#                 3: the rejected flat-load / LDS-weight flag bits refused;
#                 4: + fedagg_finalize_f64, fedagg_reduce_rows_ref (fp64 / bf16 /
#                    fp16 keys of the generic aggregator);
#                 5: + fedagg_rows_plan (which kernel a borrowed-rows call takes);
#                 6: + fedagg_host_mapped (page-locked host operands in place)
FEDAGG_INIT = 0x1
FEDAGG_FINALIZE = 0x2
FEDAGG_NT = 0x4
FEDAGG_SCALAR = 0x8
FEDAGG_DTYPE_BF16 = 1
FEDAGG_DTYPE_F16 = 2
FEDAGG_DTYPE_F64 = 3
FEDAGG_UNROLL_SHIFT = 8
FEDAGG_VPT_SHIFT = 12
FEDAGG_BS_SHIFT = 14
FEDAGG_MAP_SHIFT = 18
FEDAGG_FAST = 0x200000
FEDAGG_RELU = 0x400000
FEDAGG_CONV_GATHER = 0x800000
FEDAGG_POOL_PLANES = 0x1000000
FEDAGG_CONV_MAXPOOL2 = 0x2000000
FEDAGG_CONV_POOL_PAD1 = 0x4000000
FEDAGG_EINVAL = -22
# fedagg_rows_plan kinds
FEDAGG_ROWS_NARROW1 = 1
FEDAGG_ROWS_NARROW2 = 2
FEDAGG_ROWS_NARROW4 = 3
FEDAGG_ROWS_WIDE = 4
FEDAGG_ROWS_TILE4x8 = 5
FEDAGG_ROWS_TILE8x4 = 6
FEDAGG_ROWS_SPLITK = 7
FEDAGG_ROWS_FLAT = 8

FEDAGG_ALGO_FEDAVG = 0
FEDAGG_ALGO_ADABEST = 1
FEDAGG_ALGO_FEDDYN = 2


class SgdParams(ctypes.Structure):
    """struct fedagg_sgd_params (include/fedagg.h)."""

    _fields_ = [
        ("neg_lr", ctypes.c_float),
        ("momentum", ctypes.c_float),
        ("one_minus_dampening", ctypes.c_float),
        ("weight_decay", ctypes.c_float),
        ("nesterov", ctypes.c_int),
        ("maximize", ctypes.c_int),
    ]


class StepArgs(ctypes.Structure):
    """struct fedagg_step_args (include/fedagg.h)."""

    _fields_ = [
        ("algo", ctypes.c_int),
        ("coef", ctypes.c_float),
        ("cloud", ctypes.c_void_p),
        ("aux", ctypes.c_void_p),
        ("avg_prev", ctypes.c_void_p),
        ("momentum_buf", ctypes.c_void_p),
        ("momentum_init", ctypes.c_int),
        ("grad_out", ctypes.c_void_p),
        ("avg_out", ctypes.c_void_p),
        ("sgd", SgdParams),
    ]


class Conv2dShape(ctypes.Structure):
    """struct fedagg_conv2d_shape (include/fedagg.h)."""

    _fields_ = [(n, ctypes.c_int64) for n in
                ("M", "C", "H", "W", "OC", "KH", "KW", "stride_h", "stride_w", "pad_h", "pad_w",
                 "OH", "OW")]


class PoolArgs(ctypes.Structure):
    """struct fedagg_pool_args (include/fedagg.h)."""

    _fields_ = ([(n, ctypes.c_int64) for n in
                 ("N", "C", "H", "W", "pad_top", "pad_bottom", "pad_left", "pad_right",
                  "lrn_size")]
                + [(n, ctypes.c_float) for n in ("lrn_alpha", "lrn_beta", "lrn_k")]
                + [("flags", ctypes.c_int32)]
                + [(n, ctypes.c_int64) for n in
                   ("pool_kh", "pool_kw", "pool_sh", "pool_sw", "pool_ph", "pool_pw")])


# (name, restype, argtypes) for every symbol include/fedagg.h declares.
SIGNATURES = {
    "fedagg_abi_version": (ctypes.c_int, []),
    "fedagg_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "fedagg_column_mapping": (
        ctypes.c_int,
        [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    ),
    "fedagg_rows_plan": (
        ctypes.c_int,
        [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
    ),
    "fedagg_reduce_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
         ctypes.c_int, ctypes.c_void_p],
    ),
    "fedagg_reduce_rows_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
         ctypes.c_void_p],
    ),
    "fedagg_reduce_blocked_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
         ctypes.c_void_p],
    ),
    "fedagg_pack_row_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_void_p],
    ),
    "fedagg_host_mapped": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "fedagg_pack_segments_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p],
    ),
    "fedagg_unpack_row_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_void_p, ctypes.c_void_p],
    ),
    "fedagg_teacher_linear_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
    ),
    "fedagg_teacher_conv2d_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(Conv2dShape), ctypes.c_void_p,
         ctypes.c_int, ctypes.c_void_p],
    ),
    "fedagg_conv_stage": (ctypes.c_int, [ctypes.c_int64]),
    "fedagg_conv_order": (ctypes.c_int, [ctypes.POINTER(Conv2dShape), ctypes.c_int]),
    "fedagg_conv_pool_fusable": (ctypes.c_int, [ctypes.POINTER(Conv2dShape), ctypes.c_int]),
    "fedagg_pool_output": (
        ctypes.c_int,
        [ctypes.POINTER(PoolArgs), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
         ctypes.POINTER(ctypes.c_int64)],
    ),
    "fedagg_pad_lrn_maxpool_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(PoolArgs), ctypes.c_void_p, ctypes.c_void_p],
    ),
    "fedagg_finalize_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_float, ctypes.c_int64, ctypes.c_void_p,
         ctypes.c_void_p],
    ),
    "fedagg_reduce_rows_ref": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
    ),
    "fedagg_finalize_f64": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_void_p,
         ctypes.c_void_p],
    ),
    "fedagg_fedavg_sgd_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_int64, ctypes.c_void_p],
    ),
    "fedagg_adabest_sgd_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p],
    ),
    "fedagg_server_step_f32": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
         ctypes.POINTER(SgdParams), ctypes.c_int64, ctypes.c_void_p],
    ),
    "fedagg_reduce_step_blocked_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
         ctypes.POINTER(StepArgs), ctypes.c_void_p],
    ),
    "fedagg_reduce_step_rows_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
         ctypes.c_float, ctypes.c_int, ctypes.POINTER(StepArgs), ctypes.c_void_p],
    ),
    "fedagg_feddyn_sgd_f32": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p],
    ),
}

_lock = threading.Lock()
_lib = None


class FedAggError(RuntimeError):
    """A libfedagg call returned a non-zero status."""


def _hip_runtimes_mapped():
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return paths


def load():
    """Load (once) and return the ctypes handle; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise FedAggError(
                f"{LIB_PATH} not found: build it with `python -c "
                f"'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
            )
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        # the version first: a library built before an entry point existed
        # must fail with this message, not at the symbol lookup
        lib.fedagg_abi_version.restype = ctypes.c_int
        lib.fedagg_abi_version.argtypes = []
        built = lib.fedagg_abi_version()
        if built != ABI_VERSION:
            raise FedAggError(f"{LIB_PATH} has ABI version {built}, this package needs "
                              f"{ABI_VERSION}; rebuild the library")
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                raise FedAggError(f"{LIB_PATH} does not export {name}; rebuild the library") \
                    from None
            fn.restype = res
            fn.argtypes = args
        runtimes = _hip_runtimes_mapped()
        if len(runtimes) > 1:
            raise FedAggError(
                "two HIP runtimes are mapped (%s); import torch before fedsim_amd"
                % sorted(runtimes)
            )
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().fedagg_strerror(rc).decode()
        raise FedAggError(f"{what} failed ({rc}): {msg}")


def exported_symbols():
    """Names of the C-ABI entry points (the ones include/fedagg.h declares)."""
    return list(SIGNATURES)
