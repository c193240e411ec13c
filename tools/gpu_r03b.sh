#!/bin/bash
# Round 3: new FedDF / config tests first, then the whole GPU suite, smoke,
# the bench line and the FedDF teacher bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_feddf_cnn.py tests/test_gpu_feddf_teachers.py tests/test_gpu_configs.py \
    -k "fused or feddf_cnn or fallback or reused or configs_ or simplecnn or mismatch" > "$OUT/pytest_new.log" 2>&1 \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 600 python tools/bench_feddf_teachers.py --K 100,1000 > "$OUT/feddf_teachers.jsonl" 2> "$OUT/feddf_teachers.err"
rc=$?
echo "exit $rc"
exit $rc
