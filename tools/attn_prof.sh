#!/bin/bash
# attention parity tests + rocprof of tools/bench_attn.py (HIP path only) -> gpurun_out/pattn
set -e
bash scripts_gpu_round.sh attn
export TMPDIR=/tmp
HIP_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pattn -o run --output-format csv -- python3 tools/bench_attn.py > gpurun_out/pattn.log 2>&1
