#!/bin/bash
# Full GPU test suite (one process) + smoke + 1-GPU headline bench; logs under gpurun_out/r2.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_full.txt 2>&1
rc=$?
tail -3 gpurun_out/r2/gpu_full.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2/smoke.txt 2>&1 || { tail -5 gpurun_out/r2/smoke.txt; exit 1; }
tail -1 gpurun_out/r2/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r2/bench_default.txt 2>&1 || { tail -5 gpurun_out/r2/bench_default.txt; exit 1; }
tail -1 gpurun_out/r2/bench_default.txt
