#!/bin/bash
# zoo GPU tests, then ResNeXt / ShuffleNet / Inception throughput vs stock
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_zoo_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/zoo_gpu_tests.txt 2>&1
rc=$?
echo "zoo tests rc=$rc" >> gpurun_out/zoo_gpu_tests.txt
tail -3 gpurun_out/zoo_gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
ZOO_CFGS="resnext50_32x4d 224 256;shufflenet_v2_x1_0 224 256;inception_v3 299 128" bash tools/gpu_zoo_bench.sh
