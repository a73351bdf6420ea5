#!/bin/bash
# Full GPU suite, then the ResNet-50 bench with the data-grad path variants on one box
# (MIPIPE_DGRAD_FWD = 1 default / 2 with 1x1 stride-1 / 0 gather kernels), then the per-call profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/full_iter_tests.txt 2>&1 || { tail -40 $O/full_iter_tests.txt; exit 1; }
tail -2 $O/full_iter_tests.txt
for m in 1 2 0 1; do
  MIPIPE_DGRAD_FWD=$m timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 > $O/ab_bench_$m.txt 2>&1 || { tail -20 $O/ab_bench_$m.txt; exit 1; }
  echo "MIPIPE_DGRAD_FWD=$m $(tail -1 $O/ab_bench_$m.txt | cut -c1-200)"
done
bash $R/tools/r2/gpu_percall.sh
