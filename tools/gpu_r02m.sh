#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02m}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
