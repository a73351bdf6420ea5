set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 400 python -u bench.py --force-reduce > gpurun_out/r5_fr_r50.txt 2> gpurun_out/r5_fr_r50.err || { tail -30 gpurun_out/r5_fr_r50.err; exit 1; }
echo done
