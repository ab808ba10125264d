#!/bin/bash
# attention tests + HIP-only timing for the default build and an A/B variant .so ($1)
set -e
bash scripts_gpu_round.sh attn
HIP_ONLY=1 timeout -k 10 200 python3 tools/bench_attn.py > gpurun_out/attn_a.log 2>&1
SWH_LIB_PATH=$1 HIP_ONLY=1 timeout -k 10 200 python3 tools/bench_attn.py > gpurun_out/attn_b.log 2>&1
