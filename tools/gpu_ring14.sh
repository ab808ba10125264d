set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -q -x -k "ring14 or fused_sampler" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_ring14_tests.log 2>&1 || { tail -30 gpurun_out/r3_ring14_tests.log; exit 1; }
tail -2 gpurun_out/r3_ring14_tests.log
timeout -k 10 300 python -u tools/env_ab.py SWH_LM_RING14 1 0 > gpurun_out/r3_ring14_ab.log 2>&1 || { tail -20 gpurun_out/r3_ring14_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_ring14_ab.log
