set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 400 python -u bench.py --deterministic 1 --tune 2 --save-tune $O/r5_r50_det_table.json --reference-config off --time-deterministic off > $O/r5_r50_tablegen.txt 2>&1 || exit 1
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 400 python -u bench.py --model bert_base --seq 128 --deterministic 1 --tune 2 --save-tune $O/r5_bert_det_table.json > $O/r5_bert_tablegen.txt 2>&1 || exit 1
echo done
