set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "silu_rows or act_frag or fragw" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_gu_tests.log 2>&1 || { tail -30 gpurun_out/r3_gu_tests.log; exit 1; }
tail -2 gpurun_out/r3_gu_tests.log
timeout -k 10 300 python -u tools/gu_ab.py > gpurun_out/r3_gu_ab.log 2>&1 || { tail -20 gpurun_out/r3_gu_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_gu_ab.log
