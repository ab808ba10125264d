set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench_v6.json 2> gpurun_out/bench_v6.err || { tail -20 gpurun_out/bench_v6.err; exit 1; }
timeout -k 10 120 python -u tools/bench_decode.py 2>&1 | grep -v amdgpu.ids > gpurun_out/bdec6.log || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof6 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof6.log 2>&1 || { tail -20 gpurun_out/prof6.log; exit 1; }
f=$(find /tmp/prof6 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r2_v6_bench_kernel_stats.csv
