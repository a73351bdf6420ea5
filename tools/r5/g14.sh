set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_crop_ab2.txt $O/r5_crop_ab_bf16.txt
REF="--model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --reference-config off --time-deterministic off"
bash tools/r5/env_ab.sh $O/r5_crop_ab2.txt 2 MIPIPE_TAP_CROP=0 MIPIPE_TAP_CROP=1 -- $REF || exit 1
bash tools/r5/env_ab.sh $O/r5_crop_ab_bf16.txt 2 MIPIPE_TAP_CROP=0 MIPIPE_TAP_CROP=1 -- --model resnet18 --res 32 --batch 1024 --reference-config off --time-deterministic off || exit 1
timeout -k 10 300 python -u bench.py > $O/r5_bench_default.txt 2> $O/r5_bench_default.err || exit 1
echo done
