#!/bin/bash
# fused stem: numerics tests, stem micro A/B, bench A/B, per-call profile of the fused stem
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_stem_fused_gpu.py > $O/g_stem_tests.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|^E  .*(assert|Error)" $O/g_stem_tests.txt | cut -c1-200 | head -30
if [ $rc -gt 1 ]; then tail -30 $O/g_stem_tests.txt; exit 1; fi
timeout -k 10 300 python3 tools/r3/stem_ab.py > $O/g_stem_ab.txt 2>&1 || { tail -30 $O/g_stem_ab.txt; exit 1; }
cat $O/g_stem_ab.txt
for i in 1 2; do
  MIPIPE_STEM_FUSED=1 timeout -k 10 300 python3 bench.py --steps 30 > $O/g_bench_on_$i.txt 2>&1 || { tail -20 $O/g_bench_on_$i.txt; exit 1; }
  tail -1 $O/g_bench_on_$i.txt | cut -c1-160
  MIPIPE_STEM_FUSED=0 timeout -k 10 300 python3 bench.py --steps 30 > $O/g_bench_off_$i.txt 2>&1 || { tail -20 $O/g_bench_off_$i.txt; exit 1; }
  tail -1 $O/g_bench_off_$i.txt | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_g -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/g_prof.txt 2>&1 || { tail -20 $O/g_prof.txt; exit 1; }
cd $R
T=$(ls $O/prof_g/*/run_kernel_trace.csv $O/prof_g/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/g_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/g_stats.txt
rm -rf $O/prof_g
head -12 $O/g_stats.txt
grep -E "stem|splitk" $O/g_calls.txt | head -20
