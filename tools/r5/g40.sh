#!/bin/bash
# wgrad3x3 fp32-atomic output (no workspace sum) — tests under the switch + same-box A/B
set -o pipefail
mkdir -p gpurun_out
MIPIPE_WGRAD3_ATOMIC=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad3x3_gpu.py > gpurun_out/g40_tests.txt 2>&1 || { tail -30 gpurun_out/g40_tests.txt; exit 1; }
tail -2 gpurun_out/g40_tests.txt
for r in 1 2 3; do
  MIPIPE_WGRAD3_ATOMIC=0 timeout -k 10 200 python bench.py --steps 30 --warmup 10 >> gpurun_out/g40_ab.txt 2>/dev/null && echo "A(ws) done" &&
  MIPIPE_WGRAD3_ATOMIC=1 timeout -k 10 200 python bench.py --steps 30 --warmup 10 >> gpurun_out/g40_ab.txt 2>/dev/null && echo "B(atomic) done" || exit 1
done
python -c "import json;[print(json.loads(l)['value']) for l in open('gpurun_out/g40_ab.txt') if l.startswith('{')]"
cd /tmp && export TMPDIR=/tmp && MIPIPE_WGRAD3_ATOMIC=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g40prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/g40_prof.log 2>&1
