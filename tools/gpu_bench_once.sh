set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r3_v4b_bench.json 2> gpurun_out/r3_v4b_bench.err || { tail -20 gpurun_out/r3_v4b_bench.err; exit 1; }
tail -c 200 gpurun_out/r3_v4b_bench.json
