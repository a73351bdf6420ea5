#!/bin/bash
# Tile-config correctness + ResNet-50 per-layer sweep of every config.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/tile_tests.txt 2>&1 || { tail -40 gpurun_out/r2/tile_tests.txt; exit 1; }
tail -2 gpurun_out/r2/tile_tests.txt
timeout -k 10 600 python -u tools/tile_sweep.py --batch 256 --iters 10 > gpurun_out/r2/tile_sweep_r50.jsonl 2>&1 || { tail -5 gpurun_out/r2/tile_sweep_r50.jsonl; exit 1; }
tail -1 gpurun_out/r2/tile_sweep_r50.jsonl
