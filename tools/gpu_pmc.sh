set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- python3 tools/bench_decode.py > gpurun_out/pmcf.log 2>&1 || { tail -5 gpurun_out/pmcf.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw -o run -- python3 tools/bench_decode.py > gpurun_out/pmcw.log 2>&1 || { tail -5 gpurun_out/pmcw.log; exit 1; }
du -sh gpurun_out/pmcf gpurun_out/pmcw
