#!/bin/bash
# Per-kernel times (rocprofv3 kernel trace) of the teacher batches with the
# buffer-descriptor Linear kernel and with the generic one.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03j}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/buf" -o buf -- python3 tools/bench_feddf_teachers.py --K 1000 --no-vmap --reps 5 > "$OUT/buf.log" 2>&1 \
&& FEDAGG_LIB=tools/variants/libfedagg_tlgeneric.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gen" -o gen -- python3 tools/bench_feddf_teachers.py --K 1000 --no-vmap --reps 5 > "$OUT/gen.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
