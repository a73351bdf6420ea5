#!/bin/bash
# fp32 (reference precision) path: kernel numerics vs float64, ResNet-18 CIFAR fp32 bench vs stock.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/fp32_tests.txt 2>&1 || { tail -40 gpurun_out/r2/fp32_tests.txt; exit 1; }
tail -3 gpurun_out/r2/fp32_tests.txt
timeout -k 10 300 python bench.py --model resnet18 --res 32 --batch 1024 --dtype fp32 --steps 30 --warmup 5 > gpurun_out/r2/bench_r18_fp32.txt 2>&1 || { tail -20 gpurun_out/r2/bench_r18_fp32.txt; exit 1; }
tail -1 gpurun_out/r2/bench_r18_fp32.txt
timeout -k 10 300 python bench.py --model resnet18 --res 32 --batch 1024 --dtype bf16 --steps 30 --warmup 5 > gpurun_out/r2/bench_r18_bf16.txt 2>&1 || exit 1
tail -1 gpurun_out/r2/bench_r18_bf16.txt
timeout -k 10 400 python bench.py --impl stock --model resnet18 --res 32 --batch 1024 --dtype fp32 --steps 30 --warmup 5 > gpurun_out/r2/bench_r18_fp32_stock.txt 2>&1 || exit 1
tail -1 gpurun_out/r2/bench_r18_fp32_stock.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2/prof_r18_fp32 -o run -- python3 $R/bench.py --model resnet18 --res 32 --batch 1024 --dtype fp32 --steps 5 --warmup 3 > $R/gpurun_out/r2/prof_r18_fp32.txt 2>&1 || exit 1
echo prof-ok
