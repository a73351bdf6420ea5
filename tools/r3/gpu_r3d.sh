#!/bin/bash
# wgrad3x3 numerics, BERT graph diag, bench A/B (wgrad3x3 on/off), per-call profile
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad3x3_gpu.py > $O/d_w3_tests.txt 2>&1 || { tail -40 $O/d_w3_tests.txt; exit 1; }
tail -2 $O/d_w3_tests.txt
timeout -k 10 300 python3 tools/r3/bert_graph_diag.py > $O/d_bert_diag.txt 2>&1 || { tail -40 $O/d_bert_diag.txt; exit 1; }
grep -E "losses|<<<|flat grad" $O/d_bert_diag.txt | head -30
for i in 1 2; do
  MIPIPE_WGRAD3=1 timeout -k 10 300 python3 bench.py --steps 30 > $O/d_bench_w3on_$i.txt 2>&1 || { tail -20 $O/d_bench_w3on_$i.txt; exit 1; }
  tail -1 $O/d_bench_w3on_$i.txt | cut -c1-200
  MIPIPE_WGRAD3=0 timeout -k 10 300 python3 bench.py --steps 30 > $O/d_bench_w3off_$i.txt 2>&1 || { tail -20 $O/d_bench_w3off_$i.txt; exit 1; }
  tail -1 $O/d_bench_w3off_$i.txt | cut -c1-200
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py > $O/d_prod_tests.txt 2>&1 || { tail -40 $O/d_prod_tests.txt; exit 1; }
tail -2 $O/d_prod_tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_d -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/d_prof.txt 2>&1 || { tail -20 $O/d_prof.txt; exit 1; }
cd $R
T=$(ls $O/prof_d/*/run_kernel_trace.csv $O/prof_d/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/d_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/d_stats.txt
head -12 $O/d_stats.txt
grep wgrad3x3 $O/d_calls.txt | head -20
