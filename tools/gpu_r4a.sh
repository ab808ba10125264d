mkdir -p gpurun_out
timeout -k 10 400 python -u tools/row_invariance_probe.py > gpurun_out/r4_rowinv.log 2>&1; echo "probe rc=$?"
tail -30 gpurun_out/r4_rowinv.log
timeout -k 10 700 python -u -m pytest tests/test_trainer_contract_gpu.py tests/test_rewards_gpu.py tests/test_gpt2_gpu.py -v -m gpu --timeout 200 --timeout-method thread -k "contract or reward or train" > gpurun_out/r4_contract.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r4_contract.log | tail -40
exit $rc
