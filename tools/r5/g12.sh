set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 400 python -u bench.py --force-reduce > gpurun_out/r5_fr_r50.txt 2> gpurun_out/r5_fr_r50.err || { tail -30 gpurun_out/r5_fr_r50.err; exit 1; }
timeout -k 10 600 python -u tools/tile_sweep.py --model resnet18 --res 32 --batch 1024 --dtype fp32 > gpurun_out/r5_r18_fp32_sweep.jsonl 2> gpurun_out/r5_r18_fp32_sweep.err || exit 1
PROF_MARKER=sgd_kernel PROF_LAST=5 bash tools/gpu_run.sh prof r5_r18fp32 --model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --steps 10 --warmup 3 --reference-config off || exit 1
echo done
