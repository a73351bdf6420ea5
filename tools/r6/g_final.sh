#!/bin/bash
# round-6 final evidence: full -m gpu suite (no -x), smoke, default bench line, BERT bench line,
# ResNet-50 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/f3_full.txt 2>&1
echo "full rc=$?"
tail -3 $O/f3_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/f3_smoke.txt 2>&1 || exit 1
echo smoke ok
timeout -k 10 600 python -u bench.py > $O/f3_bench.jsonl 2> $O/f3_bench.err || exit 1
cut -c1-300 $O/f3_bench.jsonl
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 > $O/f3_bert.jsonl 2> $O/f3_bert.err || exit 1
cut -c1-300 $O/f3_bert.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_f3_r50 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_f3_r50.log 2>&1 || exit 1
echo done
