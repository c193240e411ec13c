#!/bin/bash
# HBM traffic of the FedDF teacher kernels (SimpleCNN2 layers at K=500) with
# the XCD-aware tile order (the product library) and without it
# (tools/variants/libfedagg_noxcd.so, -DFEDAGG_CONV_XCD_ORDER=0): one
# FETCH_SIZE and one WRITE_SIZE pass each, the calibration passes, and a
# timing A/B of the two builds interleaved in one process.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03pmc}
mkdir -p "$OUT"
pmc() {  # pmc <counter> <dir> <cmd...>
  local c=$1 d=$2
  shift 2
  timeout -s KILL 300 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/$d" -o "$d" -- "$@" \
    > "$OUT/$d.log" 2>&1
}
AB="tools/ab_teacher_conv.py --K 500 --rounds 1 --iters 1"
pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
&& pmc WRITE_SIZE calib_write ./tools/pmc_calib \
&& pmc FETCH_SIZE teach_fetch python3 $AB fedsim_amd/libfedagg.so \
&& pmc WRITE_SIZE teach_write python3 $AB fedsim_amd/libfedagg.so \
&& pmc FETCH_SIZE noxcd_fetch python3 $AB tools/variants/libfedagg_noxcd.so \
&& pmc WRITE_SIZE noxcd_write python3 $AB tools/variants/libfedagg_noxcd.so \
&& timeout -k 10 600 python3 tools/ab_teacher_conv.py fedsim_amd/libfedagg.so tools/variants/libfedagg_noxcd.so --K 500 --rounds 3 --iters 5 > "$OUT/ab_xcd.jsonl" 2> "$OUT/ab_xcd.err"
rc=$?
echo "exit $rc"
exit $rc
