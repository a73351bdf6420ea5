#!/bin/bash
# fused-epilogue stores through a sink (no store behind a branch): numerics, ResNet-50 bench, per-call trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zi
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_stem_fused_gpu.py tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py -k "dgrad or conv or stem or pool or det or production or bn" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/r50_$i.txt 2>&1 || { tail -20 $O/r50_$i.txt; exit 1; }
  echo "r50 $(tail -1 $O/r50_$i.txt | cut -c60-130)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pr -o run -- python3 $R/bench.py --steps 3 --warmup 4 > $O/pr.txt 2>&1 || { tail -20 $O/pr.txt; exit 1; }
cd $R
T=$(ls $O/pr/*/run_kernel_trace.csv $O/pr/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/r50_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 14 > $O/r50_stats.txt
rm -rf $O/pr
head -3 $O/r50_stats.txt
grep -c conv_fwd_kernel $O/r50_calls.txt | cut -c1-110
