set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_step_parity_gpu.py \
  "tests/test_engine_gpu.py::test_early_exit_stops_when_every_row_finished" \
  "tests/test_engine_gpu.py::test_fp32_greedy_matches_transformers_fp32_generate" \
  "tests/test_engine_gpu.py::test_checkpoint_resume_is_bit_identical_and_loads_in_transformers" \
  tests/test_ppo_gpu.py tests/test_dp_gpu.py -k "not bench_launches" > gpurun_out/t1.log 2>&1
