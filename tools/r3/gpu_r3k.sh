#!/bin/bash
# Round 3 re-entry check on a rebuilt tree: headline bench, smoke, full GPU suite, kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 bench.py --steps 30 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | cut -c1-300
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/prof.txt 2>&1 || { tail -20 $O/prof.txt; exit 1; }
cd $R
T=$(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/stats.txt
rm -rf $O/prof
head -20 $O/stats.txt
