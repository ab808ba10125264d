set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -k "attention" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -2 $O/k.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "shared_prompt or hip_attention or step_matches or prefix or cfg5 or fork or bf16" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/m.log 2>&1 || { tail -40 $O/m.log; exit 1; }
tail -2 $O/m.log
timeout -k 10 300 python -u tools/train_kernels.py --reps 3 > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
grep "ms per training" $O/train.log
