"""CPU-side checks of the C-ABI boundary: libfedagg.so loads into torch's HIP
runtime, exports every entry point include/fedagg.h declares, its constants
match the Python mirror, and argument validation rejects bad calls before any
device work (no GPU needed for any of this)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "fedagg.h")
LIB = os.path.join(REPO, "fedsim_amd", "libfedagg.so")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fedagg_[a-z0-9_]+)\s*\(", text)))


def header_defines():
    out = {}
    for m in re.finditer(r"#define\s+(FEDAGG_[A-Z0-9_]+)\s+\(?(-?0x[0-9A-Fa-f]+|-?\d+)\)?",
                         open(HEADER).read()):
        out[m.group(1)] = int(m.group(2), 0)
    return out


@pytest.fixture(scope="module")
def lib():
    import torch  # noqa: F401
    from fedsim_amd import _native

    return _native.load()


def test_header_declares_the_abi():
    fns = header_functions()
    assert fns == sorted([
        "fedagg_abi_version", "fedagg_strerror", "fedagg_column_mapping", "fedagg_reduce_f32",
        "fedagg_reduce_rows_f32", "fedagg_rows_plan", "fedagg_host_mapped",
        "fedagg_reduce_blocked_f32", "fedagg_pack_row_f32", "fedagg_pack_segments_f32",
        "fedagg_unpack_row_f32", "fedagg_teacher_linear_f32", "fedagg_teacher_conv2d_f32",
        "fedagg_conv_stage", "fedagg_conv_order", "fedagg_conv_pool_fusable", "fedagg_pool_output",
        "fedagg_pad_lrn_maxpool_f32",
        "fedagg_finalize_f32", "fedagg_finalize_f64", "fedagg_reduce_rows_ref",
        "fedagg_fedavg_sgd_f32",
        "fedagg_adabest_sgd_f32", "fedagg_feddyn_sgd_f32", "fedagg_server_step_f32",
        "fedagg_reduce_step_blocked_f32", "fedagg_reduce_step_rows_f32",
    ])


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for fn in header_functions():
        assert fn in exported, fn
        assert hasattr(lib, fn)


def test_python_mirror_matches_header(lib):
    from fedsim_amd import _native

    d = header_defines()
    assert _native.ABI_VERSION == d["FEDAGG_ABI_VERSION"] == lib.fedagg_abi_version()
    for name in ("FEDAGG_INIT", "FEDAGG_FINALIZE", "FEDAGG_NT", "FEDAGG_SCALAR",
                 "FEDAGG_UNROLL_SHIFT", "FEDAGG_VPT_SHIFT", "FEDAGG_MAP_SHIFT", "FEDAGG_EINVAL",
                 "FEDAGG_RELU", "FEDAGG_CONV_GATHER", "FEDAGG_POOL_PLANES", "FEDAGG_CONV_MAXPOOL2",
                 "FEDAGG_CONV_POOL_PAD1"):
        assert getattr(_native, name) == d[name], name
    assert set(_native.exported_symbols()) == set(header_functions())


def test_single_hip_runtime(lib):
    from fedsim_amd import _native

    assert len(_native._hip_runtimes_mapped()) == 1


def test_argument_validation_without_device(lib):
    E = -22
    null = None
    # negative sizes
    assert lib.fedagg_reduce_f32(null, 0, null, -1, 4, null, null, 1.0, 1, null) == E
    assert lib.fedagg_reduce_f32(null, 0, null, 1, -4, null, null, 1.0, 1, null) == E
    # missing output / weights / rows / accumulator
    assert lib.fedagg_reduce_f32(16, 4, 16, 1, 4, null, null, 1.0, 1, null) == E
    assert lib.fedagg_reduce_f32(16, 4, null, 1, 4, null, 16, 1.0, 1, null) == E
    assert lib.fedagg_reduce_f32(null, 4, 16, 1, 4, null, 16, 1.0, 1, null) == E
    assert lib.fedagg_reduce_f32(16, 4, 16, 1, 4, null, 16, 1.0, 0, null) == E  # no INIT, no acc
    assert lib.fedagg_reduce_f32(16, 2, 16, 1, 4, null, 16, 1.0, 1, null) == E  # ldx < P
    assert lib.fedagg_reduce_f32(16, 4, 16, 1, 4, null, 16, 1.0, 1 | 0x800000, null) == E
    assert lib.fedagg_reduce_f32(16, 1 << 31, 16, 1, (1 << 30) + 1, null, 16, 1.0, 1, null) == E
    assert lib.fedagg_reduce_rows_f32(null, 16, 1, 4, null, 16, 1.0, 1, null) == E
    assert lib.fedagg_finalize_f32(null, 1.0, 4, 16, null) == E
    assert lib.fedagg_finalize_f32(16, 1.0, -1, 16, null) == E
    assert lib.fedagg_fedavg_sgd_f32(16, 1.0, 17, null, 4, null) == E  # misaligned
    assert lib.fedagg_adabest_sgd_f32(16, 0.6, 1.0, 16, null, null, 4, null) == E
    # fused reduce + step: missing / malformed step operands
    from fedsim_amd import _native

    sgd = _native.SgdParams(-1.0, 0.0, 1.0, 0.0, 0, 0)
    ok = _native.StepArgs(0, 0.0, 16, None, None, None, 0, None, None, sgd)
    rs = lib.fedagg_reduce_step_blocked_f32
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3, None, null) == E  # no step
    no_cloud = _native.StepArgs(0, 0.0, None, None, None, None, 0, None, None, sgd)
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3, ctypes.byref(no_cloud), null) == E
    ada_no_aux = _native.StepArgs(1, 0.6, 16, None, None, None, 0, None, None, sgd)
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3, ctypes.byref(ada_no_aux), null) == E
    mom = _native.SgdParams(-1.0, 0.9, 1.0, 0.0, 0, 0)
    no_buf = _native.StepArgs(0, 0.0, 16, None, None, None, 1, None, None, mom)
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3, ctypes.byref(no_buf), null) == E
    assert rs(16, 4, 3000, 16, 1, 4, null, 1.0, 3, ctypes.byref(ok), null) == E  # bad C
    assert rs(16, 4, 4096, 16, 5, 4, null, 1.0, 3, ctypes.byref(ok), null) == E  # B > Kcap
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3 | 0x10000, ctypes.byref(ok), null) == E
    assert rs(16, 1 << 18, 4096, 16, 1, 4, null, 1.0, 3, ctypes.byref(ok), null) == E  # 4 GiB
    misaligned = _native.StepArgs(0, 0.0, 20, None, None, None, 0, None, None, sgd)
    assert rs(16, 4, 4096, 16, 1, 4, null, 1.0, 3, ctypes.byref(misaligned), null) == E
    rr = lib.fedagg_reduce_step_rows_f32
    assert rr(16, 16, 1, 4, null, 1.0, 3, None, null) == E  # no step
    assert rr(null, 16, 1, 4, null, 1.0, 3, ctypes.byref(ok), null) == E  # no row table
    assert rr(16, 16, 1, 4, null, 1.0, 2, ctypes.byref(ok), null) == E  # no INIT, no acc
    assert rr(16, 16, 1, 4, null, 1.0, 3 | 0x8, ctypes.byref(ok), null) == E  # SCALAR
    assert rr(16, 16, 1, 4, null, 1.0, 3, ctypes.byref(misaligned), null) == E
    assert rr(16, 16, 1, 4, null, 1.0, 3, ctypes.byref(ada_no_aux), null) == E
    assert lib.fedagg_server_step_f32(0, 16, 0.0, 16, null, null, null, 0, null, None, 4,
                                      null) == E  # no sgd params
    # P == 0 is a no-op success
    assert lib.fedagg_reduce_f32(null, 0, null, 0, 0, null, null, 1.0, 1, null) == 0
    assert lib.fedagg_finalize_f32(null, 1.0, 0, null, null) == 0
    assert lib.fedagg_strerror(E) == b"fedagg: invalid argument"
    assert lib.fedagg_strerror(0) == b"success"


def test_ops_refuse_cpu_tensors():
    import torch

    from fedsim_amd import ops

    with pytest.raises(ValueError, match="HIP device"):
        ops.reduce_slab(torch.ones(2, 3), torch.ones(2), torch.empty(3))
    with pytest.raises(TypeError, match="float32"):
        ops.finalize(torch.ones(3, dtype=torch.float64), 2)


def test_build_is_gfx950():
    out = subprocess.check_output(
        ["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
         f"--input={LIB}"], text=True, stderr=subprocess.STDOUT,
    ) if os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler") else ""
    if not out:
        raw = open(LIB, "rb").read()
        assert b"gfx950" in raw
    else:
        assert "gfx950" in out
    assert ctypes.sizeof(ctypes.c_void_p) == 8


def test_fuse_step_policy():
    """ops.fuse_step_pays: the last drain runs the server step fused except at
    2^20 <= P < 2^24 with >= 128 rows (profiles/r01bq/, r01br/, r01bs/), and
    for borrowed rows at any P >= 2^20 with >= 128 rows (r01cf/)."""
    from fedsim_amd import ops

    assert ops.fuse_step_pays(25_000_000, 1000)       # headline: fused
    assert ops.fuse_step_pays(199_210, 1000)          # narrow1 sizes: fused
    assert ops.fuse_step_pays(1_085_668, 10)          # few rows: one launch
    assert ops.fuse_step_pays(1_085_668, 127)
    assert not ops.fuse_step_pays(1_085_668, 128)     # SimpleCNN2 x 1000 clients: split
    assert not ops.fuse_step_pays((1 << 24) - 1, 1000)
    assert ops.fuse_step_pays(1 << 24, 1000)
    # borrowed rows (pointer table): split from 2^20 columns on, any size
    assert not ops.fuse_step_pays(25_000_000, 1000, borrowed=True)
    assert not ops.fuse_step_pays(1 << 20, 128, borrowed=True)
    assert ops.fuse_step_pays(25_000_000, 127, borrowed=True)
    assert ops.fuse_step_pays(199_210, 1000, borrowed=True)


def test_column_mapping_decision():
    """fedagg_column_mapping: the library's default mapping per P (narrow, one
    column per lane below 2^20, two from there on; unroll 8 / 16 / 8) and the
    forced ones; host-side, no device needed."""
    from fedsim_amd import ops

    assert ops.column_mapping(199_210) == ("narrow1", 8)
    assert ops.column_mapping(1_085_668) == ("narrow2", 16)
    assert ops.column_mapping(25_000_000) == ("narrow2", 8)
    assert ops.column_mapping(125_000_000, B=64) == ("narrow4", 8)  # short launches
    assert ops.column_mapping(125_000_000, B=65) == ("narrow2", 8)
    assert ops.column_mapping(125_000_000, B=100) == ("narrow2", 8)  # profiles/r01bo/
    assert ops.column_mapping(1_085_668, B=100) == ("narrow2", 16)
    assert ops.column_mapping(25_000_000, max_vw=1) == ("narrow1", 8)
    assert ops.column_mapping(25_000_001) == ("narrow1", 8)  # odd P: one column per lane
    assert ops.column_mapping(8, ops.tuning_flags(mapping="narrow4")) == ("narrow4", 8)
    assert ops.column_mapping(6, ops.tuning_flags(mapping="narrow4")) == ("narrow2", 8)
    assert ops.column_mapping(25_000_000, ops.tuning_flags(mapping="wide")) == ("wide", None)
    assert ops.column_mapping(8, ops.tuning_flags(mapping="narrow2", unroll=32)) == ("narrow2", 32)
    assert ops.column_mapping(7, ops.tuning_flags(mapping="narrow2", unroll=32)) == ("narrow1", 32)
    assert ops.column_mapping(7, ops.tuning_flags(mapping="narrow1", unroll=16)) == ("narrow1", 16)
    # unroll selectors the narrow kernels do not build fall back to the default
    assert ops.column_mapping(199_210, ops.tuning_flags(unroll=4)) == ("narrow1", 8)


def test_rows_plan_decision():
    """fedagg_rows_plan: the borrowed-rows call takes the wide per-row tiles
    only under the default flags (NT / INIT / FINALIZE allowed); any tuning
    field -- a forced mapping, k-unroll, slots per lane, block size -- keeps
    the column kernel it names, so an A/B caller measures what it asked for
    (advisor, round 5).  Host-side, no device needed."""
    from fedsim_amd import _native, ops

    base = _native.FEDAGG_NT | _native.FEDAGG_INIT | _native.FEDAGG_FINALIZE
    assert ops.rows_plan(25_000_000, 1000) == "tile4x8"
    assert ops.rows_plan(25_000_000, 1000, base) == "tile4x8"
    assert ops.rows_plan(3_000_004, 11) == "tile8x4"
    assert ops.rows_plan(1_500_000, 9) == "narrow2"        # too few workgroups for a tile
    assert ops.rows_plan(199_210, 1000) == "narrow1"
    assert ops.rows_plan(25_000_001, 1000) == "narrow1"    # odd P: no 16-B vectors
    assert ops.rows_plan(25_000_000, 1000, aligned=False) == "narrow1"
    assert ops.rows_plan(25_000_000, 0) == "narrow4"        # no rows: the tiles need one
    assert ops.rows_plan(25_000_000, 1000, _native.FEDAGG_SCALAR) == "narrow1"
    for tuned, want in ((ops.tuning_flags(mapping="narrow2"), "narrow2"),
                        (ops.tuning_flags(mapping="narrow4"), "narrow4"),
                        (ops.tuning_flags(mapping="wide"), "wide"),
                        (ops.tuning_flags(unroll=4), "narrow2"),
                        (ops.tuning_flags(vpt=2), "narrow2"),
                        (ops.tuning_flags(bs=512), "narrow2")):
        assert ops.rows_plan(25_000_000, 1000, base | tuned) == want, hex(tuned)
    assert ops.rows_plan(4096, 1000, ops.tuning_flags(fast=True)) == "splitk"
    assert ops.rows_plan(1 << 30, 2) == "flat"


def test_conv_and_pool_host_side_shapes(lib):
    """The host-only helpers of the FedDF conv / pool kernels: the conv's LDS
    stage depth, and the pool pass's output size (torch's floor-mode
    max_pool2d formula) and its rejections (no device access)."""
    import ctypes

    from fedsim_amd import _native, ops

    assert [lib.fedagg_conv_stage(r) for r in (0, 1, 16, 17, 32, 75, 96, 1600)] == \
        [0, 16, 16, 32, 32, 16, 32, 32]
    # which chain order (kernel) a conv takes: SimpleCNN2's conv2 goes to the
    # LDS-resident kernel in chunks of 4 channels; its 3-channel conv1 (and
    # any 1- or 3-channel 3x3 / 5x5 stride-1 conv) to the LDS-resident kernel
    # with every channel staged, which keeps the (c, kh, kw) chain, as do a
    # strided conv, a 7x7 kernel and the gather flag
    same = (2, 2, 2, 2)
    assert ops.conv_order((64, 3, 24, 24), 64, (5, 5), (1, 1), same) == 0
    assert ops.conv_order((64, 1, 28, 28), 32, (5, 5), (1, 1), same) == 0
    assert ops.conv_order((64, 2, 24, 24), 64, (5, 5), (1, 1), same) == 2
    assert ops.conv_order((64, 64, 12, 12), 64, (5, 5), (1, 1), same) == 2
    # SimpleCNN's conv2: chunks of 4 would need 16 staging registers, so 2
    assert ops.conv_order((64, 32, 14, 14), 64, (5, 5), (1, 1), (1, 1, 1, 1)) == 2
    assert ops.conv_order((64, 64, 12, 12), 64, (5, 5), (1, 1), same, gather=True) == 0
    assert ops.conv_order((64, 64, 12, 12), 64, (5, 5), (2, 2), same) == 0
    assert ops.conv_order((64, 64, 12, 12), 64, (7, 7), (1, 1), (3, 3, 3, 3)) == 0
    assert ops.conv_order((64, 4, 40, 40), 8, (5, 5), (1, 1), same) == 0  # tile past the LDS plan
    # SimpleCNN2 (simple_models.py:245-252): 24x24 -> pad 25x25 -> pool 3/2 -> 12x12; 12 -> 13 -> 6
    a = ops.pool_args((64, 64, 24, 24), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0))
    assert ops.pool_output(a) == (12, 12)
    a = ops.pool_args((64, 64, 12, 12), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0))
    assert ops.pool_output(a) == (6, 6)
    # SimpleCNN (simple_models.py:157): max_pool2d(2, 2, padding=1) on 28x28 -> 15x15
    assert ops.pool_output(ops.pool_args((1, 32, 28, 28), pool=(2, 2, 2, 2, 1, 1))) == (15, 15)
    assert ops.pool_output(ops.pool_args((1, 3, 5, 7), (1, 2, 3, 4))) == (8, 14)  # no pool
    oh, ow, cb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    a = ops.pool_args((8, 64, 24, 24), (0, 1, 0, 1), None, (3, 3, 2, 2, 0, 0))
    assert lib.fedagg_pool_output(ctypes.byref(a), ctypes.byref(oh), ctypes.byref(ow),
                                  ctypes.byref(cb)) == 0
    assert cb.value * 625 * 4 <= 40960 and cb.value >= 1  # padded planes within 40 KiB of LDS
    for bad in (ops.pool_args((1, 1, 200, 200)),                         # plane > 64 KiB
                ops.pool_args((1, 1, 8, 8), pool=(2, 2, 2, 2, 2, 0)),    # padding > kernel / 2
                ops.pool_args((1, 1, 2, 2), pool=(3, 3, 1, 1, 0, 0)),    # kernel > input
                ops.pool_args((1, 1, 8, 8), (-1, 0, 0, 0)),
                ops.pool_args((1, 1 << 24, 16, 8))):                     # image >= 2^31 floats
        assert lib.fedagg_pool_output(ctypes.byref(bad), ctypes.byref(oh), ctypes.byref(ow),
                                      ctypes.byref(cb)) == _native.FEDAGG_EINVAL


def test_struct_layouts_match_the_header(tmp_path):
    """Every struct include/fedagg.h declares has the same size and field
    offsets in the ctypes binding as in C (compiled here with gcc against the
    header), e.g. fedagg_pool_args' flags in the former padding after lrn_k."""
    import ctypes
    import shutil
    import subprocess

    from fedsim_amd import _native

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {
        "fedagg_pool_args": _native.PoolArgs,
        "fedagg_conv2d_shape": _native.Conv2dShape,
        "fedagg_sgd_params": _native.SgdParams,
        "fedagg_step_args": _native.StepArgs,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fedagg.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for field, _ in py._fields_:
            lines.append(f'  printf("{cname} {field} %zu\\n", offsetof({cname}, {field}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(ln.split()[:2]): int(ln.split()[2]) for ln in out if ln.strip()}
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for field, _ in py._fields_:
            assert got[(cname, field)] == getattr(py, field).offset, (cname, field)


def test_stale_library_fails_with_the_version_message(tmp_path, monkeypatch):
    """A libfedagg.so built against an older header (ABI 1: before the
    FedDF / slab-row entry points) is refused with the version message before
    any symbol lookup, rather than failing on the first missing entry point."""
    from fedsim_amd import _native

    src = tmp_path / "old.c"
    src.write_text("int fedagg_abi_version(void) { return 1; }\n")
    so = tmp_path / "libfedagg_old.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)])
    monkeypatch.setattr(_native, "LIB_PATH", str(so))
    monkeypatch.setattr(_native, "_lib", None)
    with pytest.raises(_native.FedAggError, match="ABI version 1, this package needs %d" % _native.ABI_VERSION):
        _native.load()


def test_rejected_ab_flag_bits_are_gone():
    """The flat-load / LDS-weight A/B switches (flag bits 0x10000 / 0x20000,
    measured and rejected) are no longer part of the ABI: the
    header reserves the bits and the Python side no longer names them."""
    import re

    from fedsim_amd import _native, ops

    hdr = open(os.path.join(REPO, "include", "fedagg.h")).read()
    assert not re.search(r"#define FEDAGG_(FLAT|LDSW)\b", hdr)
    assert not hasattr(_native, "FEDAGG_FLAT") and not hasattr(_native, "FEDAGG_LDSW")
    import inspect

    assert "flat" not in inspect.signature(ops.tuning_flags).parameters
    src = open(os.path.join(REPO, "fedsim_amd", "csrc", "fedagg_kernels.hip")).read()
    # no build-variant knob of a finished experiment is left in the kernels
    assert not re.search(r"^\s*#\s*if(n?def)?\b", src, re.M), "A/B build knobs in the kernels"


def test_build_is_reproducible():
    """The library is built with a fixed compilation-unit id, so identical
    sources and flags give a byte-identical library (the md5 that keys
    bench.py's PMC summary survives a rebuild).  tools/repro_build.py builds
    twice from copies in different directories and records the md5s."""
    import json

    import __graft_entry__ as G

    assert any(f.startswith("-cuid=") for f in G.HIP_FLAGS)
    with open(os.path.join(REPO, "profiles", "r05_repro_build.json")) as f:
        rec = json.load(f)
    assert rec["identical"] and rec["builds"][0]["md5"] == rec["builds"][1]["md5"]
    assert rec["builds"][0]["dir"] != rec["builds"][1]["dir"]
    assert rec["flags"] == G.HIP_FLAGS


def test_reduce_rows_ref_rejects_bad_arguments():
    """fedagg_reduce_rows_ref validates before any HIP call (none is made
    here: no GPU): an unknown dtype, negative sizes, INIT without rows, flags
    it does not take, missing pointers -> FEDAGG_EINVAL; P = 0 is a no-op."""
    from fedsim_amd import _native

    lib = _native.load()
    f = lib.fedagg_reduce_rows_ref
    E, INIT, BF16, F64 = (_native.FEDAGG_EINVAL, _native.FEDAGG_INIT,
                          _native.FEDAGG_DTYPE_BF16, _native.FEDAGG_DTYPE_F64)
    p = 4096  # a pointer value: never dereferenced on these paths
    bad = [
        (0, p, p, 1, 8, None, p, INIT),            # dtype 0
        (4, p, p, 1, 8, None, p, INIT),            # dtype past the last code
        (BF16, p, p, 1, -1, None, p, INIT),        # P < 0
        (BF16, p, p, -1, 8, p, p, 0),              # B < 0
        (F64, p, p, 0, 8, None, p, INIT),          # INIT with no rows
        (BF16, p, p, 1, 8, None, p, INIT | _native.FEDAGG_FINALIZE),  # flag it does not take
        (BF16, p, p, 1, 8, None, None, INIT),      # no out
        (BF16, p, p, 1, 8, None, p, 0),            # continuing without acc_in
        (BF16, None, p, 1, 8, None, p, INIT),      # rows missing
        (F64, p, None, 1, 8, None, p, INIT),       # weights missing
        (0, p, p, 1, 0, None, p, INIT),            # unknown dtype even at P = 0
    ]
    for args in bad:
        assert f(*args, None) == E, args
    assert f(BF16, p, p, 1, 0, None, p, INIT, None) == 0  # P = 0: nothing to do
