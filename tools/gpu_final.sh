set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_final.log 2>&1 || { tail -30 gpurun_out/gpu_final.log; exit 1; }
tail -1 gpurun_out/gpu_final.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -c 200 gpurun_out/bench_final.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof8 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof8.log 2>&1 || { tail -20 gpurun_out/prof8.log; exit 1; }
f=$(find /tmp/prof8 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r2_v8_bench_kernel_stats.csv
