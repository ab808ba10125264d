set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_step_parity_gpu.py -k "bf16 or cfg5" \
  "tests/test_dp_gpu.py::test_dp_resume_restores_each_rank_state" > gpurun_out/t2.log 2>&1
timeout -k 10 120 python -u tools/attn_probe.py --step 128 --reps 3 > gpurun_out/attn_probe.log 2>&1
timeout -k 10 120 python -u tools/attn_probe.py --step 255 --reps 2 >> gpurun_out/attn_probe.log 2>&1
