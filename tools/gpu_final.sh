set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_final.log 2>&1 || { tail -30 gpurun_out/gpu_final.log; exit 1; }
tail -1 gpurun_out/gpu_final.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -c 200 gpurun_out/bench_final.json
