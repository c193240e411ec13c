"""ISA guard for the exact-mode kernels of libfedagg.so (CPU-only: the gfx950
code object is extracted and disassembled here, nothing runs on a GPU).

The bitwise contract with the reference rests on two roundings per client
term -- ``value * weight`` then ``sum_v + new_v`` (fedsim/utils/
aggregators.py:21,40) -- and on IEEE true division at get / pop (:60,122).
``-ffp-contract=off`` keeps the source's mul / add apart, but round 5 found a
fold it does not cover: ``fptrunc(x * w)`` to fp16 became ``v_fma_mixlo_f16``
(one rounding of the exact product), caught only by a rare tie.  This test
inspects what the compiler emitted, per kernel instance:

* ``k_reduce_rows_ref<RefF16 | RefBf16>``: no mixed-precision or f16 FMA
  (``v_fma_mix*``, ``v_mad_mix*``, ``v_fma_f16``, ``v_fmac_f16``,
  ``v_pk_fma_f16``, ``v_mad_f16``);
* every exact-mode reduce / finalize instance -- ``k_reduce_narrow`` and
  ``k_reduce_vec`` with the EpiStore epilogue, every ``k_reduce_rows_ref``
  (f32 / f16 / bf16 / f64), ``k_finalize`` / ``k_finalize_f64``: each FMA-class
  instruction (f32, f64, packed or mixed) lies inside an IEEE divide
  expansion (``v_div_scale`` ... ``v_div_fixup``) or is a 64-bit integer
  division step (its literal is one of the 2^32 scaling constants);
* the fused reduce + server step (EpiStep) instances: FMAs are the SGD
  step's explicit ``__builtin_fmaf`` terms and the divide's, which run
  after the client loop -- none may sit in an innermost loop that loads
  client rows (a vector load and no divide), i.e. in the reduction itself.

FEDAGG_FAST's split-K kernels sum with fmaf by design (normwise mode) and
are not checked.  Run as a script on another build to check it:
``python tests/test_isa_guard.py path/to/libfedagg.so``.
"""
import collections
import os
import re
import shutil
import subprocess
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "fedsim_amd", "libfedagg.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

FMA = re.compile(r"^(v_fma_\w+|v_fmac_\w+|v_pk_fma_\w+|v_mad_mix\w*|v_mad_f16\w*|v_mad_f32\w*"
                 r"|v_mac_\w+|v_fmaak_\w+|v_fmamk_\w+|v_madak_\w+|v_madmk_\w+|v_pk_mad_f16)$")
HALF_FMA = re.compile(r"^(v_fma_mix\w*|v_mad_mix\w*|v_fma_f16\w*|v_fmac_f16\w*|v_pk_fma_f16"
                      r"|v_mad_f16\w*|v_pk_mad_f16)$")
# the u64 division expansion scales through f32 by 2^32 / 2^-32 / -2^32 / 2^64
INT_DIV_LITERALS = ("0x4f800000", "0x2f800000", "0xcf800000", "0x5f800000", "0x4f7ffffe")
LOAD = re.compile(r"^(buffer_load|global_load|flat_load)")
BRANCH = re.compile(r"^s_(c)?branch")
FUNC = re.compile(r"^([0-9a-f]{16}) <(.+)>:$")
INSN = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-F]{12}):")
TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>\s*$")


def disassemble(lib: str) -> str:
    """The gfx950 code object of ``lib``, disassembled (demangled).
    ``llvm-objdump --offloading`` writes the bundles next to its input, so
    it runs on a copy in a temporary directory."""
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([OBJDUMP, "--offloading", so], cwd=d, check=True, capture_output=True)
        co = [f for f in os.listdir(d) if f.endswith("gfx950")]
        assert len(co) == 1, os.listdir(d)
        return subprocess.run([OBJDUMP, "-d", "-C", "--no-show-raw-insn",
                               os.path.join(d, co[0])], check=True, capture_output=True,
                              text=True).stdout


def parse(text: str):
    """{function: [(addr, mnemonic, operands, branch_target or None)]}"""
    funcs = collections.OrderedDict()
    cur = base = None
    for line in text.splitlines():
        m = FUNC.match(line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            funcs[cur] = []
            continue
        m = INSN.match(line)
        if cur is None or not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if BRANCH.match(op):
            t = TARGET.search(line)
            if t and t.group(1) == cur:
                tgt = base + int(t.group(2), 16)
        funcs[cur].append((addr, op, args.strip(), tgt))
    return funcs


def divide_windows(ins):
    """Index spans of IEEE divide expansions: each is two v_div_scale and
    one v_div_fixup (f32 or f64); interleaved divides form one span."""
    spans, depth, start = [], 0.0, None
    for i, (_, op, _, _) in enumerate(ins):
        if op.startswith("v_div_scale"):
            if depth <= 0:
                start = i
            depth += 0.5
        elif op.startswith("v_div_fixup"):
            depth -= 1
            if depth <= 0 and start is not None:
                spans.append((start, i))
                start, depth = None, 0.0
    return spans


def innermost_loops(ins):
    """Address spans [target, branch] of backward branches containing no
    other such span."""
    loops = [(t, a) for a, _, _, t in ins if t is not None and t <= a]
    return [(t, a) for t, a in loops
            if not any((t2, a2) != (t, a) and t <= t2 and a2 <= a for t2, a2 in loops)]


def client_row_loops(ins):
    """Instruction lists of the innermost loops that read client rows: a
    vector memory load and no IEEE divide (the divide and the server step
    run once per column after the client loop; their loops load the step's
    operands next to a divide)."""
    out = []
    for t, a in innermost_loops(ins):
        body = [x for x in ins if t <= x[0] <= a]
        if any(LOAD.match(op) for _, op, _, _ in body) and \
                not any(op.startswith("v_div_scale") for _, op, _, _ in body):
            out.append(body)
    return out


def kind(name: str):
    """Which rule a kernel instance falls under (None: not checked)."""
    if "k_reduce_splitk" in name:
        return None  # FEDAGG_FAST: fmaf partial sums by design
    if "k_reduce_rows_ref<" in name:
        return "rows_ref"
    if ("k_reduce_narrow<" in name or "k_reduce_vec<" in name):
        if "EpiStore" in name:
            return "exact"
        if "EpiStep<" in name:
            return "step"
    if re.search(r"k_finalize(_f64)?\(", name):
        return "exact"
    return None


def violations(funcs):
    """(problems, instances checked per rule)."""
    bad, seen = [], collections.Counter()
    for name, ins in funcs.items():
        k = kind(name)
        if k is None:
            continue
        seen[k] += 1
        if k == "rows_ref" and ("RefF16" in name or "RefBf16" in name):
            seen["rows_ref_half"] += 1
            for _, op, args, _ in ins:
                if HALF_FMA.match(op):
                    bad.append((name, op, args, "mixed / f16 FMA in an fp16 / bf16 key"))
        if k in ("exact", "rows_ref"):
            spans = divide_windows(ins)
            for i, (_, op, args, _) in enumerate(ins):
                if FMA.match(op) and not any(a <= i <= b for a, b in spans) and \
                        not any(c in args for c in INT_DIV_LITERALS):
                    bad.append((name, op, args, "FMA outside an IEEE divide"))
        if k == "step":
            for body in client_row_loops(ins):
                for _, op, args, _ in body:
                    if FMA.match(op) or HALF_FMA.match(op):
                        bad.append((name, op, args, "FMA in the client-row loop"))
    return bad, seen


@pytest.fixture(scope="module")
def funcs():
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not available")
    return parse(disassemble(LIB))


def test_exact_kernels_have_no_contracted_arithmetic(funcs):
    bad, seen = violations(funcs)
    assert not bad, "\n".join("%s: %s %s (%s)" % (n[:140], op, a, why) for n, op, a, why in bad[:20])
    # the rules saw what they claim to guard (not vacuous)
    assert seen["exact"] >= 100 and seen["step"] >= 50, seen
    assert seen["rows_ref"] >= 20 and seen["rows_ref_half"] >= 12, seen


def test_divide_windows_are_found(funcs):
    """The analysis recognises the divides: a narrow kernel with EpiStore
    has one IEEE f32 divide per column it finalizes per lane (columns per
    lane x row pieces), five FMAs each, and the f64 finalize an f64
    divide."""
    narrow = [n for n in funcs if "k_reduce_narrow<" in n and "EpiStore" in n]
    assert narrow
    for n in narrow:
        vw = int(re.search(r"k_reduce_narrow<\d+, (\d+),", n).group(1))
        pieces = int(re.search(r"EpiStore, (\d+)>\(", n).group(1))  # row pieces per lane
        fix = sum(1 for _, op, _, _ in funcs[n] if op == "v_div_fixup_f32")
        fmas = sum(1 for _, op, _, _ in funcs[n] if FMA.match(op))
        assert fix == vw * pieces and fmas == 5 * fix, (n[:120], fix, fmas)
    f64 = [n for n in funcs if "k_finalize_f64(" in n]
    assert f64 and any(op == "v_div_fixup_f64" for _, op, _, _ in funcs[f64[0]])


def test_step_loops_are_found(funcs):
    """Every fused-step instance has an innermost loop that loads client
    rows (the rule above inspects it), and the step's own FMAs exist
    outside it (the explicit fmaf terms of the SGD update)."""
    for n, ins in funcs.items():
        if kind(n) != "step":
            continue
        assert client_row_loops(ins), n[:120]
        assert any(FMA.match(op) for _, op, _, _ in ins), n[:120]


if __name__ == "__main__":
    found, counts = violations(parse(disassemble(sys.argv[1] if len(sys.argv) > 1 else LIB)))
    for n, op, a, why in found:
        print("%s\n    %s %s  (%s)" % (n[:160], op, a, why))
    print("checked:", dict(counts), "violations:", len(found))
    sys.exit(1 if found else 0)
