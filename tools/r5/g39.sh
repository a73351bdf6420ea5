#!/bin/bash
# stem forward: y stored by the statistics pass, pool from y — tests + same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem_fused_gpu.py tests/test_model_gpu.py > gpurun_out/g39_tests.txt 2>&1 || { tail -30 gpurun_out/g39_tests.txt; exit 1; }
tail -3 gpurun_out/g39_tests.txt
for r in 1 2; do
  MIPIPE_STEM_Y_FROM_STATS=0 timeout -k 10 200 python bench.py --steps 30 --warmup 10 >> gpurun_out/g39_ab.txt 2>/dev/null && echo "A(old) done" &&
  MIPIPE_STEM_Y_FROM_STATS=1 timeout -k 10 200 python bench.py --steps 30 --warmup 10 >> gpurun_out/g39_ab.txt 2>/dev/null && echo "B(new) done" || exit 1
done
cat gpurun_out/g39_ab.txt | python -c "import sys,json;[print(json.loads(l)['value']) for l in sys.stdin if l.startswith('{')]"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g39prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/g39_prof.log 2>&1
