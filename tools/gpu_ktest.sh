#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ktest}
mkdir -p "$OUT"
for K in 250 500 750 1000; do
  timeout -k 10 300 python tools/sweep_reduce.py --K $K --rounds 3 --blocked 4096 --only-default > "$OUT/k$K.jsonl" 2>&1 || exit 1
done
timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2>/dev/null
echo "exit $?"
