#!/bin/bash
# Second half of the round-3 evidence (tools/gpu_r03_evidence.sh runs the GPU
# suite, smoke, bench, rocprof and PMC): config-4 / config-5 modes, the plugin
# round, ingest and the FedDF teacher bench.  Summaries under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03end}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --mode strong --no-cpu-baseline > "$OUT/bench_strong.json" 2> "$OUT/bench_strong.err" \
&& timeout -k 10 300 python bench.py --mode allreduce --no-cpu-baseline > "$OUT/bench_allreduce.json" 2> "$OUT/bench_allreduce.err" \
&& timeout -k 10 400 python tools/bench_plugin_round.py --headline --reps 3 > "$OUT/plugin_round.jsonl" 2> "$OUT/plugin_round.err" \
&& timeout -k 10 300 python tools/bench_ingest.py > "$OUT/ingest.json" 2> "$OUT/ingest.err" \
&& timeout -k 10 400 python tools/bench_feddf_teachers.py > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
