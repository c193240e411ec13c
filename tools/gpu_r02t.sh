#!/bin/bash
# pool pass with hoisted loads: teacher-layer GPU tests, per-layer timing, SimpleCNN2 teacher bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02t}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 200 python tools/ab_teacher_conv.py --K 500 > "$OUT/layers.jsonl" 2> "$OUT/layers.err" \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN2 > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
