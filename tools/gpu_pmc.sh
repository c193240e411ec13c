#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only alongside) for
# the bench's reduce kernel, plus the HBM read-stream ceiling microbench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2> "$OUT/hbm_peak.err" \
&& timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch \
     -- python bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1 \
&& timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write \
     -- python bench.py $ARGS > "$OUT/pmc_write.log" 2>&1 \
&& python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --K 1000 --P 25000000 \
     --flags 260 --layout blocked4096 --step fused --out "$OUT/pmc_traffic.json"
rc=$?
echo "exit $rc"
exit $rc
