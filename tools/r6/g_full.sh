#!/bin/bash
# full -m gpu suite (no -x), smoke, default bench line, reference-config profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > $O/r6_full.txt 2>&1
echo "full rc=$?"
tail -3 $O/r6_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r6_smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/r6_bench.jsonl 2> $O/r6_bench.err || exit 1
cat $O/r6_bench.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_ref4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --steps 5 --warmup 5 --reference-config off --time-deterministic off > $O/p_ref4.log 2>&1 || exit 1
echo done
