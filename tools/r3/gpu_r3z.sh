#!/bin/bash
# 3x3 depthwise forward with unconditional tap loads: zoo numerics, MobileNetV2 / ShuffleNetV2 throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_zoo_gpu.py tests/test_fp32_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for m in mobilenet_v2 shufflenet_v2_x1_0; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 > $O/$m.txt 2>&1 || { tail -20 $O/$m.txt; exit 1; }
  echo "$m $(tail -1 $O/$m.txt | cut -c60-120)"
done
