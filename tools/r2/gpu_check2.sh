#!/bin/bash
# Full GPU tests + benches (tuned vs heuristic tiles) after the main-loop generalisation.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/gpu_tests2.txt 2>&1 || { tail -30 gpurun_out/r2/gpu_tests2.txt; exit 1; }
tail -2 gpurun_out/r2/gpu_tests2.txt
for t in 1 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --tune $t > gpurun_out/r2/bench_r50_tune$t.txt 2>&1 || exit 1
  tail -1 gpurun_out/r2/bench_r50_tune$t.txt
done
timeout -k 10 300 python bench.py --model resnet18 --res 32 --batch 1024 --dtype fp32 --steps 30 --warmup 5 > gpurun_out/r2/bench_r18_fp32_t.txt 2>&1 || exit 1
tail -1 gpurun_out/r2/bench_r18_fp32_t.txt
