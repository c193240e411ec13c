#!/bin/bash
# Proves tests/test_isa_guard.py can fail: builds libfedagg.so once with the
# fp16 product's register barrier removed (fedagg_kernels.hip RefF16::prod,
# the round-5 v_fma_mixlo_f16 fold) into a scratch directory and runs the
# guard on it.  Expected: the guard reports violations (exit 1) on the mutant
# and none (exit 0) on the in-tree library.  CPU only; nothing in the repo
# is modified.
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
W="$(mktemp -d)"
trap 'rm -rf "$W"' EXIT
mkdir -p "$W/a/b"
cp -r "$REPO/include" "$W/"
sed 's|        asm("" : "+v"(q));|        /* barrier removed */|' \
    "$REPO/fedsim_amd/csrc/fedagg_kernels.hip" > "$W/a/b/k.hip"
n=$(grep -c "barrier removed" "$W/a/b/k.hip")
[ "$n" -eq 2 ] || { echo "expected 2 barriers, found $n"; exit 2; }
(cd "$W/a/b" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
    -fPIC -shared -Wall -cuid=fedagg -o "$W/lib_nobarrier.so" k.hip)
python3 "$REPO/tests/test_isa_guard.py" "$REPO/fedsim_amd/libfedagg.so" | tail -1
if python3 "$REPO/tests/test_isa_guard.py" "$W/lib_nobarrier.so" > "$W/out.txt"; then
    echo "FAIL: the guard passed a build without the barrier"; exit 1
fi
grep -c "v_fma_mix" "$W/out.txt" | sed 's/^/mutant: v_fma_mix* violations: /'
tail -1 "$W/out.txt"
echo "OK: the guard rejects the mutant"
