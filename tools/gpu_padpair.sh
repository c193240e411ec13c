#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-padpair}
mkdir -p "$OUT"
for K in 1000 750; do
  for PP in 1 8; do
    timeout -k 10 300 python tools/sweep_reduce.py --K $K --rounds 5 --blocked 4096 --only-default --pad-pair $PP > "$OUT/k${K}_pp$PP.jsonl" 2>&1 || exit 1
  done
done
timeout -k 10 300 python tools/sweep_reduce.py --K 1000 --rounds 3 --blocked 4096 > "$OUT/k1000_all.jsonl" 2>&1
echo "exit $?"
