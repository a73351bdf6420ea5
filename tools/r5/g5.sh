set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/r5/blaslt_ref.py > gpurun_out/r5_blaslt_ref.jsonl 2>&1
echo "rc=$?"
