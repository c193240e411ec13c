#!/bin/bash
# Same box: bench kernel time vs the plugin round with slab rows; the fixed
# ingest bench (distinct HBM tensors); tests touching the pack kernels.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_rows.py tests/test_gpu_aggregator.py tests/test_gpu_borrow.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 600 python tools/bench_plugin_round.py --headline --only headline --reps 3 > "$OUT/plugin_headline.jsonl" 2> "$OUT/plugin_headline.err" \
&& timeout -k 10 300 python tools/bench_ingest.py > "$OUT/ingest.json" 2> "$OUT/ingest.err" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o plugin -- python tools/bench_plugin_round.py --headline --only headline --reps 1 > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
