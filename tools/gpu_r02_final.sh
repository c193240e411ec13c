#!/bin/bash
# End-of-round evidence: full GPU suite + smoke, bench (default line) and its
# rocprof kernel stats, the config modes, the plugin round, ingest and the
# FedDF teacher bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02z}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1 \
&& timeout -k 10 300 python bench.py --mode strong --no-cpu-baseline > "$OUT/bench_strong.json" 2> "$OUT/bench_strong.err" \
&& timeout -k 10 300 python bench.py --mode allreduce --no-cpu-baseline > "$OUT/bench_allreduce.json" 2> "$OUT/bench_allreduce.err" \
&& timeout -k 10 600 python tools/bench_plugin_round.py --headline --reps 3 > "$OUT/plugin_round.jsonl" 2> "$OUT/plugin_round.err" \
&& timeout -k 10 300 python tools/bench_ingest.py > "$OUT/ingest.json" 2> "$OUT/ingest.err" \
&& timeout -k 10 600 python tools/bench_feddf_teachers.py > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
