#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sweep4}
mkdir -p "$OUT"
A="--K 1000 --P 1085668 --rounds 3 --iters 20"
timeout -k 10 300 python tools/sweep_reduce.py $A > "$OUT/strided.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py $A --blocked 1024 > "$OUT/b1024.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py $A --blocked 2048 > "$OUT/b2048.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py $A --blocked 4096 > "$OUT/b4096.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --K 10 --P 1085668 --rounds 3 --iters 50 --blocked 1024 > "$OUT/k10_b1024.jsonl" 2>&1 \
&& timeout -k 10 300 python tools/sweep_reduce.py --K 10 --P 1085668 --rounds 3 --iters 50 > "$OUT/k10_strided.jsonl" 2>&1
echo "exit $?"
