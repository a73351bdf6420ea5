set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/r5/wgrad_sweep.py > gpurun_out/r5_wgrad_sweep.jsonl 2> gpurun_out/r5_wgrad_sweep.err &&
timeout -k 10 600 python -u tools/tile_sweep.py > gpurun_out/r5_tile_sweep.jsonl 2> gpurun_out/r5_tile_sweep.err
echo "rc=$?"
