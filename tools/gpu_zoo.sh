#!/bin/bash
# Model-zoo validation: vision.hip kernel numerics + zoo model GPU tests, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_zoo_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/zoo_gpu_tests.txt 2>&1
rc=$?
echo "zoo tests rc=$rc" >> gpurun_out/zoo_gpu_tests.txt
tail -5 gpurun_out/zoo_gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -3 gpurun_out/gpu_tests.txt
exit $rc
