#!/bin/bash
# Round 2: the new GPU tests (sharded aggregator, config-size parity), then
# bench.py's three modes at N=1 and the all-reduce mode under a one-rank
# RCCL group.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharding.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 \
&& timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_param.json" 2> "$OUT/bench_param.err" \
&& timeout -k 10 300 python bench.py --mode strong --no-cpu-baseline > "$OUT/bench_strong.json" 2> "$OUT/bench_strong.err" \
&& timeout -k 10 300 python bench.py --mode allreduce > "$OUT/bench_allreduce.json" 2> "$OUT/bench_allreduce.err" \
&& timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode allreduce --no-cpu-baseline > "$OUT/bench_allreduce_torchrun1.json" 2> "$OUT/bench_allreduce_torchrun1.err"
rc=$?
echo "exit $rc"
exit $rc
