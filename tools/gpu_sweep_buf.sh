#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sweep5}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --rounds 3 --blocked 4096 > "$OUT/b4096.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --rounds 3 --blocked 2048 > "$OUT/b2048.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --K 1000 --P 1085668 --rounds 3 --iters 20 --blocked 1024 > "$OUT/small_b1024.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --K 1000 --P 1085668 --rounds 3 --iters 20 --blocked 2048 > "$OUT/small_b2048.jsonl" 2>&1 \
&& timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2>/dev/null
echo "exit $?"
