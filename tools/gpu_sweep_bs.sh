#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sweep3}
mkdir -p "$OUT"
timeout -k 10 300 python tools/sweep_reduce.py --rounds 3 --blocked 4096 > "$OUT/b4096.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --rounds 3 --blocked 2048 > "$OUT/b2048.jsonl" 2>&1
echo "exit $?"
