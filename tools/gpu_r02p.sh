#!/bin/bash
# FedDF teacher convs + pad/LRN/pool pass: GPU tests, teacher bench, rocprof breakdown
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02p}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_feddf_teachers.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
&& timeout -k 10 300 python tools/bench_feddf_teachers.py --models SimpleCNN2,SimpleMLP > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o cnn -- python3 tools/bench_feddf_teachers.py --models SimpleCNN2 --K 1000 --reps 3 --no-vmap > "$OUT/cnn.jsonl" 2> "$OUT/cnn.err"
rc=$?
echo "exit $rc"
exit $rc
