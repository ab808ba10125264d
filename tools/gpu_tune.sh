set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp swh_trl_amd/tuning/gemm_mi355x.csv gpurun_out/gemm_tuned.csv
SWH_GEMM_TUNING=tune SWH_GEMM_TABLE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tuned.csv timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tune_run.log 2>&1 || { tail -20 gpurun_out/tune_run.log; exit 1; }
wc -l gpurun_out/gemm_tuned.csv
timeout -k 10 300 python -u tools/train_kernels.py --reps 6 2>&1 | grep half-step
SWH_GEMM_TABLE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tuned.csv timeout -k 10 300 python -u tools/train_kernels.py --reps 6 2>&1 | grep half-step
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -c 120
SWH_GEMM_TABLE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tuned.csv timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -c 120
