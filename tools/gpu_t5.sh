set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 200 python -u tools/ab_generate.py 2>&1 | grep ab_generate >> gpurun_out/ab3.log || exit 1; done
cat gpurun_out/ab3.log
timeout -k 10 300 python -u tools/gemm_eff.py > gpurun_out/gemm_eff.log 2>&1 || { tail -20 gpurun_out/gemm_eff.log; exit 1; }
cat gpurun_out/gemm_eff.log | grep -v amdgpu
