set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
REF="--model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --reference-config off --time-deterministic off"
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 300 python -u bench.py $REF --tune 2 --save-tune $O/r5_r18_f32_table2.json > $O/r5_tablegen2.txt 2>&1 || exit 1
rm -f $O/r5_flat_ab2.txt
bash tools/r5/env_ab.sh $O/r5_flat_ab2.txt 2 MIPIPE_CONV_FLATTEN=0 "MIPIPE_CONV_FLATTEN=1 MIPIPE_TUNE_TABLE=$O/r5_r18_f32_table2.json" MIPIPE_CONV_FLATTEN=1 -- $REF || exit 1
echo done
