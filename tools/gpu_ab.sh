# A/B of the shipped build against a base (tools/bench_decode.py, alternating), after
# the named GPU tests.  usage: bash tools/gpu_ab.sh "<pytest -k expr>" ["VAR=value" for the base]
# (without the second argument the base is tools/_ab/base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
BASE_ENV=${2:-SWH_LIB_PATH=$PWD/tools/_ab/base.so}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -m gpu -k "$1" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  env $BASE_ENV timeout -k 10 200 python -u tools/bench_decode.py > $O/base_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/bench_decode.py > $O/new_$i.log 2>&1 || exit 1
  echo "== base $i"; tail -1 $O/base_$i.log
  echo "== new $i"; tail -1 $O/new_$i.log
done
