set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/attn_probe.py --step 128 --reps 3 > gpurun_out/attn_probe2.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attn_decode" > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
timeout -k 10 200 python -u tools/ab_generate.py > gpurun_out/ab.log 2>&1 || exit 1
SWH_LIB_PATH=tools/_probe/libbase.so timeout -k 10 200 python -u tools/ab_generate.py >> gpurun_out/ab.log 2>&1 || exit 1
grep ab_generate gpurun_out/ab.log
for L in base new base new; do
  if [ $L = base ]; then export SWH_LIB_PATH=tools/_probe/libbase.so; else unset SWH_LIB_PATH; fi
  echo "== $L" >> gpurun_out/bdec_r3a.log
  timeout -k 10 200 python -u tools/bench_decode.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/bdec_r3a.log || exit 1
done
unset SWH_LIB_PATH
grep -E "==|attn_decode|decode_step" gpurun_out/bdec_r3a.log
