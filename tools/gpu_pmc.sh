#!/bin/bash
# PMC passes (one counter per pass, --kernel-trace only alongside) for the
# bench's fused round kernel under the default (narrow) and the wide column
# mapping, the FETCH_SIZE / WRITE_SIZE calibration for 4 / 8 / 16-B accesses
# (tools/pmc_calib), and the HBM read-stream ceiling microbench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
pmc() {  # pmc <counter> <dir> <cmd...>
  local c=$1 d=$2
  shift 2
  timeout -k 10 600 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/$d" -o "$d" -- "$@" \
    > "$OUT/$d.log" 2>&1
}
timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2> "$OUT/hbm_peak.err" \
&& pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
&& pmc WRITE_SIZE calib_write ./tools/pmc_calib \
&& pmc FETCH_SIZE pmc_fetch python bench.py $ARGS \
&& pmc WRITE_SIZE pmc_write python bench.py $ARGS \
&& pmc FETCH_SIZE pmc_fetch_wide python bench.py $ARGS --mapping wide \
&& pmc WRITE_SIZE pmc_write_wide python bench.py $ARGS --mapping wide \
&& python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --K 1000 --P 25000000 \
     --layout blocked4096 --step fused --kernel-match "k_reduce_narrow<8, 2," \
     --label "k_reduce_narrow<U=8, VW=2>" --width 2 \
     --calib-fetch "$OUT/calib_fetch" --calib-write "$OUT/calib_write" \
     --out "$OUT/pmc_traffic.json" \
&& python tools/pmc_traffic.py "$OUT/pmc_fetch_wide" "$OUT/pmc_write_wide" --K 1000 \
     --P 25000000 --layout blocked4096 --step fused --kernel-match "k_reduce_vec" \
     --label "k_reduce_vec" --width 4 \
     --calib-fetch "$OUT/calib_fetch" --calib-write "$OUT/calib_write" \
     --out "$OUT/pmc_traffic_wide.json"
rc=$?
echo "exit $rc"
exit $rc
