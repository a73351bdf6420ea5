#!/bin/bash
# two-level deterministic row sums: determinism + kernel tests, det vs default A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_determinism_gpu.py tests/test_kernels_gpu.py tests/test_zoo_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/b_def_$i.txt 2>&1 || { tail -20 $O/b_def_$i.txt; exit 1; }
  echo "default $(tail -1 $O/b_def_$i.txt | cut -c60-120)"
  timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/b_det_$i.txt 2>&1 || { tail -20 $O/b_det_$i.txt; exit 1; }
  echo "det $(tail -1 $O/b_det_$i.txt | cut -c60-120)"
done
