set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ab_generate.py > gpurun_out/ab2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab_generate.py >> gpurun_out/ab2.log 2>&1 || exit 1
SWH_LIB_PATH=tools/_probe/libbase.so timeout -k 10 200 python -u tools/ab_generate.py >> gpurun_out/ab2.log 2>&1 || exit 1
grep ab_generate gpurun_out/ab2.log
timeout -k 10 300 python -u tools/train_kernels.py --reps 3 > gpurun_out/train_k.log 2>&1 || { tail -20 gpurun_out/train_k.log; exit 1; }
head -3 gpurun_out/train_k.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trk -o run -- python3 tools/train_kernels.py --reps 3 > gpurun_out/trk.log 2>&1 || { tail -20 gpurun_out/trk.log; exit 1; }
find gpurun_out/trk -name "*.csv" | head
