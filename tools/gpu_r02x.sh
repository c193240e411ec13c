#!/bin/bash
# Pool pass with the sliding channel window: teacher-layer GPU tests and the
# per-layer A/B (slide vs per-block planes) at K=500.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02x}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 300 python tools/ab_teacher_conv.py --K 500 > "$OUT/layers.jsonl" 2> "$OUT/layers.err" \
&& timeout -k 10 400 python tools/bench_feddf_teachers.py > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
