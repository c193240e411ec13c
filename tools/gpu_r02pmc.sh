#!/bin/bash
# HBM traffic of the FedDF teacher kernels (SimpleCNN2 layers at K=500): one
# FETCH_SIZE and one WRITE_SIZE pass over tools/ab_teacher_conv.py, plus the
# 4 / 8 / 16-B calibration passes over tools/pmc_calib.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02pmc}
mkdir -p "$OUT"
pmc() {  # pmc <counter> <dir> <cmd...>
  local c=$1 d=$2
  shift 2
  timeout -s KILL 300 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/$d" -o "$d" -- "$@" \
    > "$OUT/$d.log" 2>&1
}
pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
&& pmc WRITE_SIZE calib_write ./tools/pmc_calib \
&& pmc FETCH_SIZE teach_fetch python3 tools/ab_teacher_conv.py --K 500 --rounds 1 --iters 1 \
&& pmc WRITE_SIZE teach_write python3 tools/ab_teacher_conv.py --K 500 --rounds 1 --iters 1
rc=$?
echo "exit $rc"
exit $rc
