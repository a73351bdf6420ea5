#!/bin/bash
# full GPU suite + smoke + headline bench + BERT bench on the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python3 bench.py --steps 30 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | cut -c1-250
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert128.txt 2>&1 || { tail -20 $O/bert128.txt; exit 1; }
tail -1 $O/bert128.txt | cut -c1-200
timeout -k 10 300 python3 bench.py --model bert_base --seq 512 --batch 8 --steps 20 > $O/bert512.txt 2>&1 || { tail -20 $O/bert512.txt; exit 1; }
tail -1 $O/bert512.txt | cut -c1-200
