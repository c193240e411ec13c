#!/bin/bash
# Teacher slab rows padded to 16 B (all teachers on the 16-byte staging loads): teacher tests + bench (default lib twice around the 4-byte-load build).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02x9}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --no-vmap --reps 20 > "$OUT/teachers_vec.jsonl" 2> "$OUT/teachers_vec.err" \
&& FEDAGG_LIB=tools/libfedagg_tl0.so timeout -k 10 300 python tools/bench_feddf_teachers.py --no-vmap --reps 20 > "$OUT/teachers_scalar.jsonl" 2> "$OUT/teachers_scalar.err" \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --no-vmap --reps 20 > "$OUT/teachers_vec2.jsonl" 2> "$OUT/teachers_vec2.err"
rc=$?
echo "exit $rc"
exit $rc
