#!/bin/bash
# Linear kernel variants, per-kernel times (rocprofv3 kernel trace) of the
# teacher batches at K=1000: product (buffer kernel, wide layers at 4 WG/CU),
# no LDS pad (8 WG/CU everywhere), the generic kernel.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03k}
mkdir -p "$OUT"
run() {  # run <name> [lib]
  local n=$1
  if [ -n "$2" ]; then export FEDAGG_LIB=$2; else unset FEDAGG_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_$n -o $n -- python3 tools/bench_feddf_teachers.py --K 1000 --no-vmap --reps 5 > "$OUT/$n.log" 2>&1 \
  && python3 tools/linear_trace_summary.py $(ls /tmp/tr_$n/*kernel_trace.csv | head -1) $n >> "$OUT/linear.jsonl"
}
run prod && run nopad tools/variants/libfedagg_tlnopad.so && run gen tools/variants/libfedagg_tlgeneric.so \
&& run prod2 && run gen2 tools/variants/libfedagg_tlgeneric.so
rc=$?
echo "exit $rc"
exit $rc
