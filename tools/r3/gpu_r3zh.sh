#!/bin/bash
# LayerNorm forward with unconditional loads: numerics, BERT throughput, per-call LN time
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zh
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_gpu.py -k "layernorm or bert or attention or dropout" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_$i.txt 2>&1 || { tail -20 $O/bert_$i.txt; exit 1; }
echo "bert $(tail -1 $O/bert_$i.txt | cut -c60-130)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pr -o run -- python3 $R/bench.py --model bert_base --steps 3 --warmup 4 > $O/pr.txt 2>&1 || { tail -20 $O/pr.txt; exit 1; }
cd $R
T=$(ls $O/pr/*/run_kernel_trace.csv $O/pr/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/kernel_stats.py $T --step-marker adamw --last 3 --top 12 > $O/bert_stats.txt
rm -rf $O/pr
cat $O/bert_stats.txt
