#!/bin/bash
# Slab rows: tests, the round loop and borrow suites, then the plugin round at
# the headline size (slab rows vs borrowed vectors).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02d}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_rows.py tests/test_gpu_roundloop.py tests/test_gpu_borrow.py tests/test_gpu_aggregator.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 600 python tools/bench_plugin_round.py --headline --only headline --reps 3 > "$OUT/plugin_headline.jsonl" 2> "$OUT/plugin_headline.err"
rc=$?
echo "exit $rc"
exit $rc
