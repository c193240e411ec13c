#!/bin/bash
# Final-tree check: full GPU suite, smoke, default bench line with its rocprof stats.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02check}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
