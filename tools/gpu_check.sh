#!/bin/bash
# Validation call: GPU test suite, smoke(), ResNet-50 bench (default), ResNet-18 CIFAR bench, BERT bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -5 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/bench.txt
timeout -k 10 300 python bench.py --model resnet18 --res 32 --batch 1024 > gpurun_out/bench_r18.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_r18.txt
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/bench_bert.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_bert.txt
