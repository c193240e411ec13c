#!/bin/bash
# LDS-resident teacher conv kernel: GPU tests of the teacher layers, the
# per-layer A/B against the gather kernel, and the SimpleCNN2 teacher bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02s}
mkdir -p "$OUT"
true \
&& timeout -k 10 200 python tools/ab_teacher_conv.py --K 500 > "$OUT/layers.jsonl" 2> "$OUT/layers.err" \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN2 > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
