#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02l}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_properties.py -x -q --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
