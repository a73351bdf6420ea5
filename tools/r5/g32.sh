# deterministic-mode plan tables regenerated on the final kernels (ResNet-50 b256, BERT-base b32 s128)
# and a same-box A/B of the deterministic ResNet-50 step: new table vs the shipped one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 400 python -u bench.py --deterministic 1 --tune 2 --save-tune $O/r5_r50_det_table2.json --reference-config off --time-deterministic off > $O/r5_r50_tablegen2.txt 2>&1 || exit 1
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 400 python -u bench.py --model bert_base --seq 128 --deterministic 1 --tune 2 --save-tune $O/r5_bert_det_table2.json --reference-config off --time-deterministic off > $O/r5_bert_tablegen2.txt 2>&1 || exit 1
rm -f $O/r5_det_table_ab.txt
bash tools/r5/env_ab.sh $O/r5_det_table_ab.txt 2 "MIPIPE_SHIPPED_TUNE=0 MIPIPE_TUNE_TABLE=$O/r5_r50_det_table2.json" MIPIPE_SHIPPED_TUNE=1 -- --deterministic 1 --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
bash tools/r5/env_ab.sh $O/r5_det_table_ab.txt 1 MIPIPE_SHIPPED_TUNE=1 -- --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
