#!/bin/bash
# Staggered first generation of the flat conv (FEDAGG_FLAT_STAGGER = 1 / 2 / 4
# s_sleep(127) periods per slot) vs none, SimpleCNN2 layers at K=500, all
# builds interleaved in one process.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03d}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/ab_teacher_conv.py fedsim_amd/libfedagg.so tools/variants/libfedagg_stagger1.so tools/variants/libfedagg_stagger2.so tools/variants/libfedagg_stagger4.so --K 500 --rounds 3 --iters 5 > "$OUT/ab_stagger.jsonl" 2> "$OUT/ab_stagger.err"
rc=$?
echo "exit $rc"
exit $rc
