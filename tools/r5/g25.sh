set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
bash tools/r5/pmc_ta.sh l1c2fwd 256 56 64 64 3 1 1 fwd 9 > $O/r5_pmcta_l1.txt 2>&1 || exit 1
bash tools/r5/pmc_ta.sh l3c2fwd 256 14 256 256 3 1 1 fwd 11 > $O/r5_pmcta_l3.txt 2>&1 || exit 1
bash tools/r5/pmc_ta.sh l1c3fwd 256 56 64 256 1 1 0 fwd 9 > $O/r5_pmcta_l1c3.txt 2>&1 || exit 1
echo done
