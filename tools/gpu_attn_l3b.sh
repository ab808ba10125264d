set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -q -x -k "l3" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_l3_tests.log 2>&1 || { tail -30 gpurun_out/r3_l3_tests.log; exit 1; }
tail -2 gpurun_out/r3_l3_tests.log
timeout -k 10 300 python -u tools/mall_probe.py --attn-l3 > gpurun_out/r3_attn_l3d.log 2>&1 || { tail -20 gpurun_out/r3_attn_l3d.log; exit 1; }
grep "decode step" gpurun_out/r3_attn_l3d.log
