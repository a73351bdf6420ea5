set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_ntmin_ab.txt
bash tools/r5/env_ab.sh $O/r5_ntmin_ab.txt 2 MIPIPE_NT_MIN_MB=0 MIPIPE_NT_MIN_MB=40 MIPIPE_NT_MIN_MB=120 MIPIPE_NT_MIN_MB=220 -- --reference-config off --time-deterministic off || exit 1
echo done
