#!/bin/bash
# 1x1 stride-1 data-grads through the forward kernel (MIPIPE_DGRAD_FWD=2) vs the dgrad kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
for i in 1 2; do
  MIPIPE_DGRAD_FWD=2 timeout -k 10 300 python3 bench.py --steps 30 > $O/i_fwd2_$i.txt 2>&1 || { tail -20 $O/i_fwd2_$i.txt; exit 1; }
  tail -1 $O/i_fwd2_$i.txt | cut -c1-110
  timeout -k 10 300 python3 bench.py --steps 30 > $O/i_def_$i.txt 2>&1 || { tail -20 $O/i_def_$i.txt; exit 1; }
  tail -1 $O/i_def_$i.txt | cut -c1-110
done
cd /tmp && export TMPDIR=/tmp
MIPIPE_DGRAD_FWD=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_i -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/i_prof.txt 2>&1 || { tail -20 $O/i_prof.txt; exit 1; }
cd $R
T=$(ls $O/prof_i/*/run_kernel_trace.csv $O/prof_i/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/i_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 30 > $O/i_stats.txt
rm -rf $O/prof_i
head -14 $O/i_stats.txt
sort -k2 -n -r $O/i_calls.txt | head -14 | cut -c1-150
