set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PROF_MARKER=sgd_kernel PROF_LAST=5 bash tools/gpu_run.sh prof r5_r18fp32_crop --model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --steps 10 --warmup 3 --reference-config off --time-deterministic off || exit 1
timeout -k 10 600 python -u tools/tile_sweep.py --model resnet18 --res 32 --batch 1024 --dtype fp32 > gpurun_out/r5_r18_fp32_sweep_crop.jsonl 2> gpurun_out/r5_r18_fp32_sweep_crop.err || exit 1
echo done
