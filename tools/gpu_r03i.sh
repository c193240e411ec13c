#!/bin/bash
# Buffer-descriptor Linear kernel: its bitwise tests, then the teacher bench
# with the product library and with the generic Linear kernel
# (tools/variants/libfedagg_tlgeneric.so, -DFEDAGG_TL_BUF=0), alternating.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03i}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_feddf_teachers.py -k "linear or replay or simplecnn or relu" > "$OUT/pytest_linear.log" 2>&1 \
&& for i in 1 2; do \
  timeout -k 10 300 python tools/bench_feddf_teachers.py --K 100,1000 --no-vmap > "$OUT/teachers_buf_$i.jsonl" 2> "$OUT/teachers_buf_$i.err" && \
  FEDAGG_LIB=tools/variants/libfedagg_tlgeneric.so timeout -k 10 300 python tools/bench_feddf_teachers.py --K 100,1000 --no-vmap > "$OUT/teachers_generic_$i.jsonl" 2> "$OUT/teachers_generic_$i.err" || exit 1; \
done
rc=$?
echo "exit $rc"
exit $rc
