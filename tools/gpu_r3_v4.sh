set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3_v4_bench.json 2> gpurun_out/r3_v4_bench.err || { tail -20 gpurun_out/r3_v4_bench.err; exit 1; }
tail -c 400 gpurun_out/r3_v4_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof3 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
f=$(find /tmp/prof3 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3_v4_bench_kernel_stats.csv
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_v4_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r3_v4_gpu_suite.log
exit $rc
