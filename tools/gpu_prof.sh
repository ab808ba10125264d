set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof5 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || { tail -20 gpurun_out/prof5.log; exit 1; }
f=$(find /tmp/prof5 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r2_v5_bench_kernel_stats.csv; ls -la gpurun_out
