set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# 1. PMC traffic of the shipped decode kernels (one counter per pass, kernel trace only)
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- python3 tools/bench_decode.py > gpurun_out/pmcf.log 2>&1 || { tail -5 gpurun_out/pmcf.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw -o run -- python3 tools/bench_decode.py > gpurun_out/pmcw.log 2>&1 || { tail -5 gpurun_out/pmcw.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmcf gpurun_out/pmcw gpurun_out/r3_pmc_decode.json > /dev/null || exit 1
rm -rf gpurun_out/pmcf gpurun_out/pmcw
# 2. the bench line (reads the PMC summary just written)
timeout -k 10 600 python -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
tail -c 300 gpurun_out/r3_bench.json
# 3. rocprofv3 kernel statistics of the same build and command
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof3 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
f=$(find /tmp/prof3 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3_bench_kernel_stats.csv
# 4. PPO cfg3
timeout -k 10 400 python -u tools/bench_ppo.py > gpurun_out/r3_ppo_bench.json 2> gpurun_out/r3_ppo_bench.err || { tail -20 gpurun_out/r3_ppo_bench.err; exit 1; }
cat gpurun_out/r3_ppo_bench.json
