#!/bin/bash
# SimpleCNN conv2 (C = 32, 14x14): chunks of 4 channels with 16 staging
# registers (default) vs chunks of 2 with 8 (FEDAGG_CONV_CC2_XM16 build), via
# the teacher bench, default / variant / default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02xa}
mkdir -p "$OUT"
timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/cc4.jsonl" 2> "$OUT/cc4.err" \
&& FEDAGG_LIB=tools/libfedagg_cc2.so timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/cc2.jsonl" 2> "$OUT/cc2.err" \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN --K 100,1000 --no-vmap --reps 20 > "$OUT/cc4b.jsonl" 2> "$OUT/cc4b.err"
rc=$?
echo "exit $rc"
exit $rc
