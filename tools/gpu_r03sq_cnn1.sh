#!/bin/bash
# SQ counters of SimpleCNN's conv1 + ReLU + 2x2 pool launch (flat conv, POOL)
# at K=500: two rocprofv3 --pmc passes over tools/ab_conv_shape.py.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03al}
mkdir -p "$OUT"
AB="tools/ab_conv_shape.py fedsim_amd/libfedagg.so --C 1 --H 28 --OC 32 --pad 1 --shared --pool-pad 1 --rounds 1 --iters 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq_a" -o sq_a -- python3 $AB > "$OUT/sq_a.log" 2>&1 \
&& timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq_b" -o sq_b -- python3 $AB > "$OUT/sq_b.log" 2>&1
rc=$?
echo "exit $rc"
exit $rc
