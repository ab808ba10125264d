set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# PMC traffic of the shipped decode kernels (one counter per pass, kernel trace only)
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- python3 tools/bench_decode.py > gpurun_out/pmcf.log 2>&1 || { tail -5 gpurun_out/pmcf.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw -o run -- python3 tools/bench_decode.py > gpurun_out/pmcw.log 2>&1 || { tail -5 gpurun_out/pmcw.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmcf gpurun_out/pmcw gpurun_out/r3_v4_pmc_decode.json > /dev/null || exit 1
rm -rf gpurun_out/pmcf gpurun_out/pmcw
cp gpurun_out/r3_v4_pmc_decode.json profiles/r3_pmc_decode.json
