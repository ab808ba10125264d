#!/bin/bash
# Parameterised GPU evidence runs (one gpurun call runs the steps given, in order,
# and stops at the first failure; every GPU step under its own time limit).
#   bash tools/gpu_evidence.sh <tag> <step>...
# steps:
#   suite    pytest -m gpu (whole suite, one process) + smoke()      -> <tag>_gpu_suite.log
#   sel      pytest -m gpu -k "$SEL" (a subset, one process)         -> <tag>_gpu_sel.log
#   pmc      rocprofv3 FETCH_SIZE / WRITE_SIZE passes over tools/bench_decode.py -> <tag>_pmc_decode.json
#   bench    python bench.py (default K / W, CPU baseline included)  -> <tag>_bench.json
#   prof     rocprofv3 --kernel-trace --stats of bench.py --steps 1 --warmup 1 -> <tag>_bench_kernel_stats.csv
#   decode   tools/bench_decode.py (per-kernel decode timings)       -> <tag>_decode.log
#   train    tools/train_kernels.py (training half-step)             -> <tag>_train.log
#   trace    rocprofv3 kernel trace of one training half-step + tools/critical_path.py -> <tag>_critical_path.txt
#   ppo      tools/bench_ppo.py (BASELINE config 3)                  -> <tag>_ppo_bench.json
#   llama    tools/bench_llama8b.py (Llama-3-8B shapes, 1 prompt)      -> <tag>_llama8b.json
#   llama5   tools/bench_llama8b.py at config 5's per-GPU shape        -> <tag>_llama8b_c1024.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
O=gpurun_out
fail() { echo "[$1] failed (rc=$2)"; tail -20 "$3"; exit "$2"; }
for step in "$@"; do
  echo "[$step] start $(date +%T)"
  case $step in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread \
        > $O/${tag}_gpu_suite.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" $O/${tag}_gpu_suite.log | tail -30
      [ $rc -eq 0 ] || fail suite $rc $O/${tag}_gpu_suite.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > $O/${tag}_smoke.log 2>&1 || fail smoke $? $O/${tag}_smoke.log
      tail -1 $O/${tag}_smoke.log ;;
    sel)
      timeout -k 10 600 python -u -m pytest tests -v -rP -m gpu -k "$SEL" --timeout 300 --timeout-method thread \
        > $O/${tag}_gpu_sel.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" $O/${tag}_gpu_sel.log | tail -30
      [ $rc -eq 0 ] || fail sel $rc $O/${tag}_gpu_sel.log ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run \
          -- python3 tools/bench_decode.py > $O/pmc_$c.log 2>&1 || fail pmc $? $O/pmc_$c.log
      done
      python tools/pmc_summary.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/${tag}_pmc_decode.json > /dev/null \
        || fail pmc_summary $? /dev/null
      rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE ;;
    bench)
      timeout -k 10 600 python -u bench.py > $O/${tag}_bench.json 2> $O/${tag}_bench.err \
        || fail bench $? $O/${tag}_bench.err
      tail -c 400 $O/${tag}_bench.json ;;
    prof)
      rm -rf /tmp/prof_$tag
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o run \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/${tag}_prof.log 2>&1 \
        || fail prof $? $O/${tag}_prof.log
      cp "$(find /tmp/prof_$tag -name '*kernel_stats.csv' | head -1)" $O/${tag}_bench_kernel_stats.csv
      python tools/critical_path.py "$(find /tmp/prof_$tag -name '*kernel_trace.csv' | head -1)" 330 --whole \
        > $O/${tag}_bench_critical_path.txt 2>&1 || fail critical_path $? $O/${tag}_bench_critical_path.txt ;;
    decode)
      timeout -k 10 300 python -u tools/bench_decode.py > $O/${tag}_decode.log 2>&1 || fail decode $? $O/${tag}_decode.log
      tail -15 $O/${tag}_decode.log ;;
    train)
      timeout -k 10 300 python -u tools/train_kernels.py > $O/${tag}_train.log 2>&1 || fail train $? $O/${tag}_train.log
      tail -15 $O/${tag}_train.log ;;
    trace)
      rm -rf /tmp/trace_$tag
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/trace_$tag -o run \
        -- python3 tools/train_kernels.py --reps 1 > $O/${tag}_trace.log 2>&1 || fail trace $? $O/${tag}_trace.log
      cp "$(find /tmp/trace_$tag -name '*kernel_trace.csv' | head -1)" $O/${tag}_train_trace.csv
      python tools/critical_path.py $O/${tag}_train_trace.csv 150 \
        > $O/${tag}_critical_path.txt 2>&1 || fail critical_path $? $O/${tag}_critical_path.txt
      head -40 $O/${tag}_critical_path.txt ;;
    ppo)
      timeout -k 10 400 python -u tools/bench_ppo.py > $O/${tag}_ppo_bench.json 2> $O/${tag}_ppo_bench.err \
        || fail ppo $? $O/${tag}_ppo_bench.err
      tail -c 400 $O/${tag}_ppo_bench.json ;;
    llama)
      timeout -k 10 900 python -u tools/bench_llama8b.py > $O/${tag}_llama8b.json 2> $O/${tag}_llama8b.err \
        || fail llama $? $O/${tag}_llama8b.err
      tail -c 400 $O/${tag}_llama8b.json ;;
    llama5)  # config 5's per-GPU shape: 8 prompts x G 8, P 256, C 1024, beta 0.04, 16384-token passes
      timeout -k 10 900 python -u tools/bench_llama8b.py --prompts 8 --P 256 --C 1024 --fuse-budget 16384 \
        > $O/${tag}_llama8b_c1024.json 2> $O/${tag}_llama8b_c1024.err || fail llama5 $? $O/${tag}_llama8b_c1024.err
      tail -c 600 $O/${tag}_llama8b_c1024.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
