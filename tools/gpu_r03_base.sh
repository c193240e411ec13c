#!/bin/bash
# Round-3 baseline on the inherited tree: GPU suite + smoke + default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "exit $rc"
exit $rc
