#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-padtest}
mkdir -p "$OUT"
for PAD in 0 1 3 8 24 25; do
  timeout -k 10 300 python tools/sweep_reduce.py --K 1000 --rounds 3 --blocked 4096 --only-default --kcap-pad $PAD > "$OUT/pad$PAD.jsonl" 2>&1 || exit 1
done
for PAD in 0 1; do
  timeout -k 10 300 python tools/sweep_reduce.py --K 750 --rounds 3 --blocked 4096 --only-default --kcap-pad $PAD > "$OUT/k750_pad$PAD.jsonl" 2>&1 || exit 1
done
timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2>/dev/null
echo "exit $?"
