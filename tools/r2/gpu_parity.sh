#!/bin/bash
# Production-shape kernel tests + convergence parity vs stock PyTorch-ROCm.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_production_shapes_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/prod_shapes.txt 2>&1 || { tail -30 gpurun_out/r2/prod_shapes.txt; exit 1; }
tail -2 gpurun_out/r2/prod_shapes.txt
timeout -k 10 400 python -u tools/convergence.py --arch resnet18 --res 32 --batch 256 --steps 400 --dtype bf16 > gpurun_out/r2/conv_r18_bf16.jsonl 2>&1 || { tail -5 gpurun_out/r2/conv_r18_bf16.jsonl; exit 1; }
tail -1 gpurun_out/r2/conv_r18_bf16.jsonl
timeout -k 10 400 python -u tools/convergence.py --arch resnet18 --res 32 --batch 256 --steps 400 --dtype fp32 > gpurun_out/r2/conv_r18_fp32.jsonl 2>&1 || { tail -5 gpurun_out/r2/conv_r18_fp32.jsonl; exit 1; }
tail -1 gpurun_out/r2/conv_r18_fp32.jsonl
timeout -k 10 400 python -u tools/convergence.py --arch resnet50 --res 32 --batch 256 --steps 300 --dtype bf16 --log-every 5 > gpurun_out/r2/conv_r50_bf16.jsonl 2>&1 || { tail -5 gpurun_out/r2/conv_r50_bf16.jsonl; exit 1; }
tail -1 gpurun_out/r2/conv_r50_bf16.jsonl
