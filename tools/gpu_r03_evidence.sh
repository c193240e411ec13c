#!/bin/bash
# End-of-round evidence on the final round-3 tree: GPU suite + smoke, the
# bench line and its rocprof kernel stats, the headline kernel's PMC traffic
# (FETCH_SIZE / WRITE_SIZE passes + calibration); the config-4 / config-5
# modes, plugin round, ingest and FedDF bench are tools/gpu_r03_evidence_b.sh.  Large traces stay in
# /tmp on the box; only summaries land under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03end}
mkdir -p "$OUT"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
pmc() {  # pmc <counter> <dir> <cmd...>
  local c=$1 d=$2
  shift 2
  timeout -s KILL 300 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/$d" -o "$d" -- "$@" \
    > "$OUT/$d.log" 2>&1
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03prof -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1 \
&& cp /tmp/r03prof/bench_kernel_stats.csv "$OUT/rocprof_kernel_stats.csv" \
&& pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
&& pmc WRITE_SIZE calib_write ./tools/pmc_calib \
&& pmc FETCH_SIZE pmc_fetch python bench.py $ARGS \
&& pmc WRITE_SIZE pmc_write python bench.py $ARGS \
&& python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --K 1000 --P 25000000 \
     --layout blocked4096 --step fused --kernel-match "k_reduce_narrow<8, 2," \
     --label "k_reduce_narrow<U=8, VW=2>" --width 2 \
     --calib-fetch "$OUT/calib_fetch" --calib-write "$OUT/calib_write" \
     --out "$OUT/pmc_traffic.json"
rc=$?
echo "exit $rc"
exit $rc
