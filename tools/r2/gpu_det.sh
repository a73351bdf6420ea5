#!/bin/bash
# Deterministic mode: bit-identical runs + throughput cost.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_determinism_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/det_tests.txt 2>&1 || { tail -30 gpurun_out/r2/det_tests.txt; exit 1; }
tail -2 gpurun_out/r2/det_tests.txt
for d in 1 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --deterministic $d > gpurun_out/r2/bench_r50_det$d.txt 2>&1 || exit 1
  tail -1 gpurun_out/r2/bench_r50_det$d.txt
done
timeout -k 10 300 python bench.py --model resnet18 --res 32 --batch 1024 --dtype fp32 --steps 30 --warmup 5 --deterministic 1 > gpurun_out/r2/bench_r18_fp32_det.txt 2>&1 || exit 1
tail -1 gpurun_out/r2/bench_r18_fp32_det.txt
