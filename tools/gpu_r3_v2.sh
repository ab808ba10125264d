set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/mall_probe.py > gpurun_out/r3_mall_probe.log 2>&1 || { tail -20 gpurun_out/r3_mall_probe.log; exit 1; }
cat gpurun_out/r3_mall_probe.log
bash tools/gpu_r3_v1.sh
