set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "sampler" "tests/test_engine_gpu.py::test_generation_is_run_to_run_deterministic" "tests/test_engine_gpu.py::test_early_exit_stops_when_every_row_finished" > gpurun_out/t6.log 2>&1 || { tail -40 gpurun_out/t6.log; exit 1; }
tail -3 gpurun_out/t6.log
for i in 1 2; do timeout -k 10 200 python -u tools/ab_generate.py 2>&1 | grep ab_generate >> gpurun_out/ab4.log || exit 1; done
cat gpurun_out/ab4.log
timeout -k 10 300 python -u tools/gemm_eff.py > gpurun_out/gemm_eff2.log 2>&1 || { tail -20 gpurun_out/gemm_eff2.log; exit 1; }
grep "wgrad split" gpurun_out/gemm_eff2.log
