cd $GRAFT_REPO_ROOT
PROF_MARKER=adamw_kernel PROF_LAST=5 bash tools/gpu_run.sh prof bert --model bert_base --steps 5 --warmup 5 || exit 1
PROF_MARKER=sgd_kernel PROF_LAST=5 bash tools/gpu_run.sh prof r50 --steps 5 --warmup 5 || exit 1
