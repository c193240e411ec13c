#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02j}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_roundloop.py tests/test_gpu_slab_rows.py -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
