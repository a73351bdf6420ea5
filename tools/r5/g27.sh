# half-band stem backward: stem tests, same-box A/B (MIPIPE_STEM_HALF), kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_stem_fused_gpu.py > $O/r5_stem_half_tests.txt 2>&1 || exit 1
rm -f $O/r5_stem_half_ab.txt
bash tools/r5/env_ab.sh $O/r5_stem_half_ab.txt 3 MIPIPE_STEM_HALF=1 MIPIPE_STEM_HALF=0 -- --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r5_stemhalf -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 10 --reference-config off --time-deterministic off > $O/prof_r5_stemhalf.txt 2>&1 || exit 1
echo done
