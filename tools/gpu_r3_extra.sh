set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_ppo.py > gpurun_out/r3_v3_ppo_bench.json 2> gpurun_out/r3_v3_ppo_bench.err || { tail -20 gpurun_out/r3_v3_ppo_bench.err; exit 1; }
tail -c 300 gpurun_out/r3_v3_ppo_bench.json
timeout -k 10 600 python -u tools/bench_llama8b.py --prompts 8 --P 256 --C 1024 --fuse-budget 16384 > gpurun_out/r3_llama8b_c1024_1gpu.json 2> gpurun_out/r3_llama8b.err || { tail -20 gpurun_out/r3_llama8b.err; exit 1; }
tail -c 400 gpurun_out/r3_llama8b_c1024_1gpu.json
