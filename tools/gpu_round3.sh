#!/bin/bash
# PMC traffic for the current default kernel, then tests + smoke + bench +
# rocprof stats, then the bench's process-group path rehearsed at N=1 under
# torch.distributed.run (RCCL barrier + max-over-ranks, one rank).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r01e}
TAG=$TAG bash tools/gpu_pmc.sh || exit 1
OUT=gpurun_out/$TAG
TAG=$TAG bash tools/gpu_round2.sh || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 10 --warmup 2 \
    --no-cpu-baseline > "$OUT/bench_torchrun1.json" 2> "$OUT/bench_torchrun1.err" \
&& timeout -k 10 300 python bench.py --step split --no-cpu-baseline \
    > "$OUT/bench_split.json" 2> "$OUT/bench_split.err"
rc=$?
echo "exit $rc"
exit $rc
