#!/bin/bash
# FedDF conv / pool layers of SimpleCNN2: per-layer timing (HIP events), the
# counter list of this box, and one SQ counter pass over the same layers.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02r}
mkdir -p "$OUT"
timeout -k 10 120 python tools/ab_teacher_conv.py --K 500 > "$OUT/layers.jsonl" 2> "$OUT/layers.err" \
&& (timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true) \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o sq -- python3 tools/ab_teacher_conv.py --K 500 --rounds 1 --iters 1 > "$OUT/pmc_sq.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
