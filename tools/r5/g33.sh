# kernel trace of the deterministic ResNet-50 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r5_det -o run -- python $GRAFT_REPO_ROOT/bench.py --deterministic 1 --steps 5 --warmup 10 --reference-config off --time-deterministic off > $O/prof_r5_det.txt 2>&1 || exit 1
echo done
