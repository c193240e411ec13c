#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r0*.sh
# scripts).  Runs the named steps in order, each under its own time limit,
# and stops at the first step that fails (no retries): a fault, abort, time
# limit or hang ends the call there.  Summaries land in gpurun_out/$TAG/.
#
#   gpurun -- 'TAG=r04a tools/gpu_run.sh suite smoke bench rocprof pmc'
#
# steps
#   suite            pytest -m gpu on the whole tree (what the driver runs)
#   test=<spec>      pytest -m gpu on one file / node id (tests/<spec>)
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (the driver's default line)
#   benchmode=<mode> python bench.py --mode strong|allreduce (configs 4 / 5 at N=1)
#   rocprof          rocprofv3 --kernel-trace --stats of bench.py (10 steps)
#   pmc              FETCH_SIZE / WRITE_SIZE passes of the bench kernel + the
#                    tools/pmc_calib calibration -> pmc_traffic.json (with the
#                    build's md5, read by bench.py's roofline.traffic)
#   feddf            tools/bench_feddf_teachers.py (replay vs vmap per batch)
#   py=<script args> python3 tools/<script> with arguments (',' for spaces)
#   pmcpy=<script args> FETCH_SIZE / WRITE_SIZE passes (+ the pmc_calib
#                    calibration) over python3 tools/<script> (',' for spaces;
#                    tools/pmc_rows_tiles.py reads them)
#   tpy=<script args> python3 tests/<script> (the GPU checker scripts kept with
#                    the tests: fuzz_tiles.py, debug_rows_ref.py)
#   sq=<script args> two SQ-counter passes (tools/sq_summary.py reads them)
#                    over python3 tools/<script> (',' for spaces)
#   hbm_peak         tools/hbm_peak read-stream ceiling
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-side-legs"

pmc() {  # pmc <counters> <dir> <cmd...>
  local c=$1 d=$2
  shift 2
  timeout -s KILL ${PMC_TIMEOUT:-300} rocprofv3 --pmc $c --output-format csv -d "$OUT/$d" -o "$d" -- "$@" \
    > "$OUT/$d.log" 2>&1
}

step() {
  local s=$1 arg
  echo "== $s ($(date -u +%H:%M:%S))"
  case "$s" in
    suite)
      timeout -k 10 ${SUITE_TIMEOUT:-1100} python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread --durations=15 > "$OUT/pytest_gpu.log" 2>&1 ;;
    test=*)
      arg=${s#test=}
      timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest "tests/$arg" -m gpu -x -v -s --timeout 300 \
        --timeout-method thread > "$OUT/test_$(echo "$arg" | tr '/:[]' '____').log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    benchmode=*)
      arg=${s#benchmode=}
      timeout -k 10 600 python bench.py --mode $arg --no-cpu-baseline > "$OUT/bench_$arg.json" \
        2> "$OUT/bench_$arg.err" ;;
    rocprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o bench \
        -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1 \
      && cp /tmp/prof_$TAG/bench_kernel_stats.csv "$OUT/rocprof_kernel_stats.csv" ;;
    pmc)
      pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
      && pmc WRITE_SIZE calib_write ./tools/pmc_calib \
      && pmc FETCH_SIZE pmc_fetch python bench.py $PMC_ARGS \
      && pmc WRITE_SIZE pmc_write python bench.py $PMC_ARGS \
      && python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --K 1000 --P 25000000 \
           --layout blocked4096 --step fused --kernel-match "k_reduce_narrow<8, 2," \
           --label "k_reduce_narrow<U=8, VW=2>" --width 2 \
           --calib-fetch "$OUT/calib_fetch" --calib-write "$OUT/calib_write" \
           --profile "profiles/$TAG/" --out "$OUT/pmc_traffic.json" ;;
    pmcpy=*)
      arg=${s#pmcpy=}
      arg=${arg//,/ }
      pmc FETCH_SIZE calib_fetch ./tools/pmc_calib \
      && pmc WRITE_SIZE calib_write ./tools/pmc_calib \
      && pmc FETCH_SIZE pmcpy_fetch python3 tools/$arg \
      && pmc WRITE_SIZE pmcpy_write python3 tools/$arg ;;
    feddf)
      timeout -k 10 600 python -u tools/bench_feddf_teachers.py > "$OUT/feddf_teachers.jsonl" \
        2> "$OUT/feddf_teachers.err" ;;
    py=*)
      arg=${s#py=}
      arg=${arg//,/ }
      timeout -k 10 ${PY_TIMEOUT:-600} python3 -u tools/$arg > "$OUT/py_$(echo "${arg%% *}" | tr '/.' '__').out" \
        2> "$OUT/py_$(echo "${arg%% *}" | tr '/.' '__').err" ;;
    tpy=*)
      arg=${s#tpy=}
      arg=${arg//,/ }
      timeout -k 10 ${PY_TIMEOUT:-600} python3 -u tests/$arg > "$OUT/tpy_$(echo "${arg%% *}" | tr '/.' '__').out" \
        2> "$OUT/tpy_$(echo "${arg%% *}" | tr '/.' '__').err" ;;
    sq=*)
      arg=${s#sq=}
      arg=${arg//,/ }
      pmc "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
          sq_a python3 tools/$arg \
      && pmc "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
          sq_b python3 tools/$arg ;;
    hbm_peak)
      timeout -k 10 300 ./tools/hbm_peak 32 > "$OUT/hbm_peak.json" 2> "$OUT/hbm_peak.err" ;;
    *)
      echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  step "$s"
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $s failed: exit $rc"
    exit $rc
  fi
done
echo "exit 0"
