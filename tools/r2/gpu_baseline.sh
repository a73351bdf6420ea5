#!/bin/bash
# Round-2 baseline on a fresh box: GPU tests, smoke, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r2/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r2/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r2/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/r2/bench.txt
