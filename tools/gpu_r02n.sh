#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02n}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_feddf_teachers.py tests/test_gpu_roundloop.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 600 python tools/bench_feddf_teachers.py > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
