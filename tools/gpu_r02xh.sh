#!/bin/bash
# Flat conv with 128 pixels per wave for OC <= 32 (SimpleCNN conv1): teacher
# GPU tests, then the SimpleCNN teacher bench new / previous build / new.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02xh}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_teachers.log" 2>&1 \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/new.jsonl" 2> "$OUT/new.err" \
&& FEDAGG_LIB=tools/variants/libfedagg_prev.so timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/prev.jsonl" 2> "$OUT/prev.err" \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/new2.jsonl" 2> "$OUT/new2.err"
rc=$?
echo "exit $rc"
exit $rc
