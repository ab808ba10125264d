set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SWH_LIB_PATH=$PWD/tools/_ab/base.so timeout -k 10 400 python -u bench.py --variant top_p --steps 3 --warmup 1 > $O/topp_base.log 2>&1 || { tail -5 $O/topp_base.log; exit 1; }
timeout -k 10 400 python -u bench.py --variant top_p --steps 3 --warmup 1 > $O/topp_new.log 2>&1 || { tail -5 $O/topp_new.log; exit 1; }
tail -1 $O/topp_base.log | cut -c1-200
tail -1 $O/topp_new.log | cut -c1-200
