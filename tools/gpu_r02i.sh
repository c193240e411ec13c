#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02i}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_slab_rows.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 600 python tools/bench_plugin_round.py --headline --only headline --reps 3 > "$OUT/plugin.jsonl" 2> "$OUT/plugin.err" \
&& timeout -k 10 300 python tools/profile_plugin_round.py --where device_borrow > "$OUT/profile_borrow.txt" 2>&1 \
&& timeout -k 10 300 python tools/profile_plugin_round.py --where gpu_clients > "$OUT/profile_gpu_clients.txt" 2>&1
rc=$?
echo "exit $rc"
exit $rc
