#!/bin/bash
# branch-free fused dgrad epilogue ring: numerics (dgrad fusions, production shapes), overlap test,
# bench A/B vs the previous .so (kept as _C_prev), per-call trace of the layer-1 data-grads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 250 --timeout-method thread tests/test_ddp_gpu.py -k overlaps > $O/ovl_test.txt 2>&1 || { tail -30 $O/ovl_test.txt; exit 1; }
tail -1 $O/ovl_test.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/b_new_$i.txt 2>&1 || { tail -20 $O/b_new_$i.txt; exit 1; }
  echo "new $(tail -1 $O/b_new_$i.txt | cut -c60-130)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pr -o run -- python3 $R/bench.py --steps 3 --warmup 4 > $O/pr.txt 2>&1 || { tail -20 $O/pr.txt; exit 1; }
cd $R
T=$(ls $O/pr/*/run_kernel_trace.csv $O/pr/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/r50_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 12 > $O/r50_stats.txt
rm -rf $O/pr
head -8 $O/r50_stats.txt
sort -k2 -n -r $O/r50_calls.txt | head -8 | cut -c1-120
