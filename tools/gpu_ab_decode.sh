set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "act_frag or xstream or fragw or decode_gemm or generat" > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -1 gpurun_out/t1.log
for v in 1 0 1; do
  echo "== ACT_FRAG=$v" >> gpurun_out/bdec8.log
  SWH_ACT_FRAG=$v timeout -k 10 120 python -u tools/bench_decode.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/bdec8.log || exit 1
done
