#!/bin/bash
# Pool pass step indices / squares-once; flat conv occupancy A/B (3 vs 4 waves per SIMD).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02x3}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 400 python tools/ab_teacher_conv.py --K 500 --rounds 4 > "$OUT/layers.jsonl" 2> "$OUT/layers.err"
rc=$?
echo "exit $rc"
exit $rc
