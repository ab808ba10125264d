set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "silu" tests/test_engine_gpu.py -k "silu or training_grads or hip_attention_path" > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -2 gpurun_out/t7.log
for L in base new base new; do
  if [ $L = base ]; then export SWH_LIB_PATH=tools/_probe/libbase.so; else unset SWH_LIB_PATH; fi
  echo -n "$L " ; timeout -k 10 100 python -u tools/bench_silu.py 2>&1 | grep silu_mul || exit 1
done
unset SWH_LIB_PATH
timeout -k 10 300 python -u tools/train_kernels.py --reps 3 2>&1 | grep "train_kernels" || exit 1
SWH_LIB_PATH=tools/_probe/libbase.so timeout -k 10 300 python -u tools/train_kernels.py --reps 3 2>&1 | grep "train_kernels" || exit 1
