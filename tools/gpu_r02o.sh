#!/bin/bash
# Kernel breakdown of FedDF's SimpleCNN2 teacher replay at K = 1000 (before the conv kernel)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02o}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o cnn -- python3 tools/bench_feddf_teachers.py --models SimpleCNN2 --K 1000 --reps 3 --no-vmap > "$OUT/cnn.jsonl" 2> "$OUT/cnn.err"
rc=$?
echo "exit $rc"
exit $rc
