set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_ab_buf.txt
bash tools/r5/ab_run.sh nobuf 3 $O/r5_ab_buf.txt --reference-config off --time-deterministic off || exit 1
bash tools/r5/ab_run.sh nobuf 1 $O/r5_ab_buf_bert.txt --model bert_base --seq 128 || exit 1
bash tools/r4/pmc_conv.sh r5buf_l3c2_fwd 256 14 256 256 3 1 1 fwd -1 > /dev/null 2>&1 || exit 1
bash tools/r4/pmc_gemm.sh r5buf_qkv 4096,2304,768,1,1,0 -1 > /dev/null 2>&1 || exit 1
GRAFT_REPO_ROOT=/tmp/ab_nobuf bash /tmp/ab_nobuf/tools/r4/pmc_conv.sh nobuf_l3c2_fwd 256 14 256 256 3 1 1 fwd -1 > /dev/null 2>&1 || exit 1
GRAFT_REPO_ROOT=/tmp/ab_nobuf bash /tmp/ab_nobuf/tools/r4/pmc_gemm.sh nobuf_qkv 4096,2304,768,1,1,0 -1 > /dev/null 2>&1 || exit 1
cp /tmp/ab_nobuf/gpurun_out/pmc_nobuf_l3c2_fwd/summary.txt $O/pmc_nobuf_l3c2_fwd.txt
cp /tmp/ab_nobuf/gpurun_out/pmcg_nobuf_qkv/summary.txt $O/pmcg_nobuf_qkv.txt
echo done
