set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
&& timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.log 2>&1
echo "exit $?"
