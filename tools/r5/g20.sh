# waterfall-free buffer soffsets + tail-free stages + buffer im2col weight-grad operand:
# conv kernel tests, same-box A/B against the old build, kernel trace of the new build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py -k "conv or dgrad or wgrad or gemm" > $O/r5_wf_tests.txt 2>&1 || exit 1
rm -f $O/r5_wf_ab.txt
bash tools/r5/ab_run.sh old 3 $O/r5_wf_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r5_wf -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 10 --reference-config off --time-deterministic off > $O/prof_r5_wf.txt 2>&1 || exit 1
echo done
