#!/bin/bash
# The one GPU-box recipe runner (replaces the per-experiment gpurun wrappers of rounds 1-3).
# Run from the repo root, e.g. through gpurun:
#   gpurun --timeout 900 -- 'bash tools/gpu_run.sh tests'
#   gpurun --timeout 600 -- 'bash tools/gpu_run.sh bench r50 --steps 20 --warmup 5'
#   gpurun --timeout 600 -- 'bash tools/gpu_run.sh prof bert --model bert_base --steps 5 --warmup 3 --graph off'
#   gpurun --timeout 600 -- 'bash tools/gpu_run.sh pytest tests/test_kernels_gpu.py -k gemm'
#   gpurun --timeout 300 -- 'bash tools/gpu_run.sh lab 0 5'
# Recipes (several may be chained with `+`: 'smoke+tests'):
#   smoke                  __graft_entry__.smoke()
#   tests                  pytest -m gpu (whole suite)
#   pytest ARGS...         pytest ARGS (one process, per-test timeout)
#   bench NAME ARGS...     bench.py ARGS -> gpurun_out/bench_NAME.jsonl (appends)
#   prof NAME ARGS...      rocprofv3 --kernel-trace --stats of bench.py ARGS -> gpurun_out/prof_NAME/
#                          + tools/kernel_stats.py summary gpurun_out/prof_NAME/summary.txt
#                          (PROF_MARKER=<kernel ending a step> PROF_LAST=N: the last N steps only)
#   lab [SHAPE] [ROUNDS]   tools/gemm_lab/pp_lab (built on the CPU host beforehand)
# Every GPU step runs under its own timeout; the first failing step ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # step TIMEOUT LOG CMD...
  local to=$1 log=$2
  shift 2
  timeout -k 10 "$to" "$@" > "$log" 2>&1
  local rc=$?
  tail -5 "$log"
  if [ $rc -ne 0 ]; then echo "[gpu_run] step failed rc=$rc: $*"; exit $rc; fi
}

recipe=$1
shift
IFS='+' read -ra PARTS <<< "$recipe"
for r in "${PARTS[@]}"; do
  case "$r" in
    smoke)
      step 300 "$O/smoke.txt" python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)
      step 1100 "$O/gpu_tests.txt" python3 -u -m pytest tests -m gpu -q -x --timeout 300 \
        --timeout-method thread ;;
    pytest)
      step 1100 "$O/pytest.txt" python3 -u -m pytest -q -x --timeout 300 --timeout-method thread "$@"
      exit 0 ;;
    bench)
      name=$1; shift
      timeout -k 10 600 python3 bench.py "$@" >> "$O/bench_$name.jsonl" 2> "$O/bench_$name.err"
      rc=$?
      tail -1 "$O/bench_$name.jsonl" | cut -c1-400
      if [ $rc -ne 0 ]; then tail -20 "$O/bench_$name.err"; exit $rc; fi
      exit 0 ;;
    prof)
      name=$1; shift
      P=$O/prof_$name
      mkdir -p "$P"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$P" -o run -- python3 "$R/bench.py" "$@" > "$P/bench.txt" 2>&1)
      rc=$?
      if [ $rc -ne 0 ]; then tail -20 "$P/bench.txt"; exit $rc; fi
      csv=$(find "$P" -name '*kernel_trace.csv' | head -1)
      python3 tools/kernel_stats.py "$csv" --top 40 ${PROF_MARKER:+--step-marker $PROF_MARKER} \
        ${PROF_LAST:+--last $PROF_LAST} > "$P/summary.txt" 2>&1
      head -30 "$P/summary.txt"
      continue ;;
    lab)
      step 600 "$O/pp_lab.jsonl" tools/gemm_lab/pp_lab "${1:--1}" "${2:-5}"
      cat "$O/pp_lab.jsonl"
      exit 0 ;;
    *)
      echo "unknown recipe $r"; exit 2 ;;
  esac
done
