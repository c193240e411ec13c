#!/bin/bash
# Flat conv with compact per-channel row staging (product, 4 waves/SIMD) vs
# the previous layout (libfedagg_prev.so) vs compact + 5 waves/SIMD
# (libfedagg_flatwpe5.so): the conv GPU tests, then SimpleCNN2 layers at
# K=500 interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03l}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_feddf_teachers.py tests/test_gpu_feddf_cnn.py > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 600 python3 tools/ab_teacher_conv.py fedsim_amd/libfedagg.so tools/variants/libfedagg_prev.so tools/variants/libfedagg_flatwpe5.so --K 500 --rounds 3 --iters 5 > "$OUT/ab_flat.jsonl" 2> "$OUT/ab_flat.err"
rc=$?
echo "exit $rc"
exit $rc
