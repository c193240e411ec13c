# A/B of the teacher Linear tile order: the product library (XCD-ordered) vs a FEDAGG_LINEAR_XCD_ORDER=0 build in tools/_ab/, FedDF batches at K=1000 and rocprof kernel traces (profiles/r03z/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03z; mkdir -p $OUT
for rep in 1 2; do
  for v in new lin0; do
    if [ $v = new ]; then L=fedsim_amd/libfedagg.so; else L=tools/_ab/libfedagg_lin0.so; fi
    FEDAGG_LIB=$L timeout -k 10 200 python tools/bench_feddf_teachers.py --K 1000 --no-vmap --reps 10 > $OUT/feddf_${v}_$rep.jsonl 2> $OUT/feddf_${v}_$rep.err || exit 1
  done
done
for v in new lin0; do
  if [ $v = new ]; then L=fedsim_amd/libfedagg.so; else L=tools/_ab/libfedagg_lin0.so; fi
  FEDAGG_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$v -o kt -- python tools/bench_feddf_teachers.py --K 1000 --no-vmap --reps 5 > $OUT/kt_$v.log 2>&1 || exit 1
  python tools/kernel_trace_summary.py $(ls /tmp/kt_$v/*kernel_trace.csv /tmp/kt_$v/*/*kernel_trace.csv 2>/dev/null | head -1) 40 | grep -i "linear" > $OUT/linear_$v.txt
done
echo done
