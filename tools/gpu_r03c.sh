#!/bin/bash
# Flat conv without the per-k-step "upper channels" branch (product build) vs
# the round-2 flat conv (tools/variants/libfedagg_noxcd.so has it), SimpleCNN2
# layers at K=500 interleaved; then the conv GPU tests and the teacher bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03c}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/ab_teacher_conv.py fedsim_amd/libfedagg.so tools/variants/libfedagg_r03c.so --K 500 --rounds 3 --iters 5 > "$OUT/ab_flat.jsonl" 2> "$OUT/ab_flat.err" \
&& timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_feddf_teachers.py tests/test_gpu_feddf_cnn.py > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 600 python tools/bench_feddf_teachers.py --K 1000 --no-vmap > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
