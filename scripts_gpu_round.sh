#!/bin/bash
# One GPU session: parity tests, then a short bench.  Stops at the first
# fault / abort / timeout (exit codes 124/134/137/139), never retries.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -5 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
  return 0
}
for step in "$@"; do
  case $step in
    gpu) run gpu 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
    gpuall) run gpuall 1100 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ;;
    new2) run new2 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "rewards or checkpoint or dp_ or step_parity" ;;
    newp) run newp 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -s -k "selective_log_softmax or greedy_matches" ;;
    g2) run g2 600 python -u -m pytest tests/test_gpt2_gpu.py -v -m gpu --timeout 200 --timeout-method thread ;;
    cfg1) run cfg1 300 python tools/bench_cfg1.py ;;
    wide) run wide 600 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread -k "wide_gemm or llama" ;;
    shared) run shared 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "shared_prompt or step_parity or grpo_trainer_smoke or llama_grpo or rewards or checkpoint_resume" ;;
    newt) run newt 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "step_parity or adamw or bench_launches or masked_whiten" ;;
    tune) cp swh_trl_amd/tuning/gemm_mi355x.csv gpurun_out/gemm_tuned.csv && SWH_GEMM_TUNING=tune SWH_GEMM_TABLE=gpurun_out/gemm_tuned.csv run tune 900 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
    benchtuned) SWH_GEMM_TABLE=gpurun_out/gemm_tuned.csv run benchtuned 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline ;;
    lmk) run lmk 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "lm_head or decode_gemm or sampler" --timeout 120 --timeout-method thread ;;
    decab) run dec0 300 python tools/bench_decode.py && for v in vA vB; do SWH_LIB_PATH=tools/_build/$v.so run dec_$v 300 python tools/bench_decode.py || exit 1; done ;;
    attn) run attn 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k attention --timeout 120 --timeout-method thread ;;
    benchab) SWH_ATTN=torch run bench_torchattn 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline && SWH_ATTN=hip run bench_hipattn 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    dwab) SWH_DW_SPLIT=0 run b_nosplit 600 python bench.py --steps 4 --warmup 2 --no-cpu-baseline && run b_split 600 python bench.py --steps 4 --warmup 2 --no-cpu-baseline ;;
    kern) run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu ;;
    kernx) run kernx 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x ;;
    pack) run pack 400 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread -k "wide_gemm or packed_wide or llama or recapture" && run l8d1 300 python tools/bench_llama8b_decode.py && SWH_WIDE_PACK=0 run l8d0 300 python tools/bench_llama8b_decode.py ;;
    tune8) cp swh_trl_amd/tuning/gemm_mi355x.csv gpurun_out/gemm_tuned8b.csv && SWH_GEMM_TUNING=tune SWH_GEMM_TABLE=gpurun_out/gemm_tuned8b.csv run tune8 1050 python tools/bench_llama8b.py --prompts 8 --P 256 --C 1024 --steps 1 --warmup 1 --fuse-budget 16384 ;;
    shkv) run shkv 500 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread -k "shared_prompt or attn_decode or greedy or packed_wide or recapture or fused_sampler" && run dec 300 python tools/bench_decode.py && run l8d1 300 python tools/bench_llama8b_decode.py ;;
    shkvb) run l8d1 300 python tools/bench_llama8b_decode.py && SWH_DECODE_SHARED_KV=0 run l8d0 300 python tools/bench_llama8b_decode.py && run benchq 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline ;;
    l8d) run l8d1 300 python tools/bench_llama8b_decode.py ;;
    l8dt) run wt 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu --timeout 200 --timeout-method thread -k "wide_gemm" && run l8d1 300 python tools/bench_llama8b_decode.py ;;
    splitk) run splitk 400 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu --timeout 200 --timeout-method thread -k "decode_gemm" && SWH_SWEEP_CFGS="None;1,1,2;1,1,4;2,1,2;2,1,4;4,1,2;4,1,4;4,2,2;4,2,4;1,2,2;2,2,2;2,2,4;1,1,8;4,1,8;4,4,2,0,4;4,4,4,0,4;2,2,2,0,2;2,2,4,0,2" run ksweep 400 python tools/bench_decode.py --ku ;;
    decw) SWH_WIDE_KMIN=512 run decw 300 python tools/bench_decode.py ;;
    dec) run dec 300 python tools/bench_decode.py ;;
    decsteps) run dec0 200 python tools/bench_decode.py --step 1 && run dec128 200 python tools/bench_decode.py --step 128 && run dec255 200 python tools/bench_decode.py --step 255 ;;
    ku) run ku 400 python tools/bench_decode.py --ku ;;
    dual) run dual 300 python tools/bench_decode.py --dual ;;
    sweep) run sweep 300 python tools/bench_decode.py --sweep ;;
    probe) run probe 300 python tools/gemm_probe.py ;;
    btrain) run btrain 600 python tools/bench_train.py ;;
    lat) run lat 120 python tools/latency_probe.py && HIP_FORCE_DEV_KERNARG=1 run lat1 120 python tools/latency_probe.py && HIP_FORCE_DEV_KERNARG=0 run lat0 120 python tools/latency_probe.py ;;
    profdec) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run profdec 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profdec -o run --output-format csv -- python3 tools/bench_decode.py ;;
    ppo) run ppo 600 python -m pytest tests/test_ppo_gpu.py -q -m gpu -x ;;
    ppob) run ppob 600 python tools/bench_ppo.py ;;
    engine) run engine 600 python -m pytest tests/test_engine_gpu.py -q -m gpu -x ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps 3 --warmup 2 ;;
    benchq) run benchq 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    dbg_eager) AMD_SERIALIZE_KERNEL=3 GRAPH=0 C=16 run dbg_eager 300 python tools/debug_decode.py ;;
    dbg_graph) GRAPH=1 run dbg_graph 300 python tools/debug_decode.py ;;
    serial2) AMD_SERIALIZE_KERNEL=3 SWH_TRACE=1 run serial2 500 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --layers 2 ;;
    trace2) SWH_TRACE=1 run trace2 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --layers 2 ;;
    ktrace) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run ktrace 900 rocprofv3 --kernel-trace -d gpurun_out/ktrace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
    fenceab) SWH_GEMM_FENCE=0 run b_nofence 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline && run b_fence 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline && SWH_GEMM_FENCE=0 run b_nofence2 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
    l8s) SWH_TRACE=1 run l8s 400 python tools/bench_llama8b.py --prompts 2 --P 256 --C 1024 --steps 1 --warmup 1 --fuse-budget 16384 ;;
    hangp) run hangp 150 python tools/phase_probe.py --layers 2 --B 8 --L 512 && run hangp2 150 python tools/phase_probe.py --layers 2 --B 8 --L 1280 ;;
    hangq) run hangq 120 python tools/phase_probe.py --layers 1 --B 8 --L 1280 --part lmhead && run hangq2 120 python tools/phase_probe.py --layers 1 --B 8 --L 1280 --part attn ;;
    hangs) AMD_SERIALIZE_KERNEL=3 run hangs 100 python tools/phase_probe.py --layers 1 --B 8 --L 1280 ;;
    hangt) SWH_DW_STREAM=0 SWH_ATTN_SPLIT=0 run hangt1 100 python tools/phase_probe.py --layers 2 --B 8 --L 1280 && SWH_GEMM_TUNING=off run hangt2 100 python tools/phase_probe.py --layers 2 --B 8 --L 1280 ;;
    hangf) run hangf 100 python tools/phase_probe.py --layers 2 --B 8 --L 1280 --reps 3 ;;
    l8w4) SWH_WIDE_SMAX=4 SWH_TRACE=1 run l8w4 1000 python tools/bench_llama8b.py --prompts 8 --P 256 --C 1024 --steps 1 --warmup 1 --fuse-budget 16384 ;;
    l8) SWH_TRACE=1 run l8 1000 python tools/bench_llama8b.py --prompts 8 --P 256 --C 1024 --steps 1 --warmup 1 --fuse-budget 16384 ;;
    l8k) run l8k 600 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -k "llama3_8b" --timeout 200 --timeout-method thread ;;
    tk) run tk 600 python tools/train_kernels.py ;;
    proftk) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run proftk 600 rocprofv3 --kernel-trace --stats -d gpurun_out/proftk -o run --output-format csv -- python3 tools/train_kernels.py ;;
    pmcft) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run pmcft 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcft -o run --output-format csv -- python3 tools/train_kernels.py --reps 1 ;;
    pmcwt) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run pmcwt 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcwt -o run --output-format csv -- python3 tools/train_kernels.py --reps 1 ;;
    pmcf) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run pmcf 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- python3 tools/bench_decode.py ;;
    pmcw) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && run pmcw 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python3 tools/bench_decode.py ;;
    trace) SWH_TRACE=1 run trace 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
  esac
done
