set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gemm_plans.py > gpurun_out/r5_gemm_plans_bert.jsonl 2> gpurun_out/r5_gemm_plans_bert.err || exit 1
PROF_MARKER=sgd_kernel PROF_LAST=5 bash tools/gpu_run.sh prof r5_r50 --steps 10 --warmup 3 --reference-config off --time-deterministic off || exit 1
PROF_MARKER=adamw PROF_LAST=5 bash tools/gpu_run.sh prof r5_bert --model bert_base --seq 128 --steps 10 --warmup 3 || exit 1
echo done
