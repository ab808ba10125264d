set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -q -x -k "kmajor or lm_head or fused_sampler or fragw" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_kmajor_tests.log 2>&1 || { tail -30 gpurun_out/r3_kmajor_tests.log; exit 1; }
tail -2 gpurun_out/r3_kmajor_tests.log
timeout -k 10 300 python -u tools/lm_kmajor_ab.py > gpurun_out/r3_kmajor_ab.log 2>&1 || { tail -20 gpurun_out/r3_kmajor_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_kmajor_ab.log
