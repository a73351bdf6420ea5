set -e
cd $GRAFT_REPO_ROOT
for s in 0 2 3 4 5 6 7 8 9 10 11; do timeout -k 10 120 tools/gemm_lab/pp_lab $s 5 >> gpurun_out/pp1.jsonl; done
cat gpurun_out/pp1.jsonl
