set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r3_bench_env_ab.log
: > $o
for v in "X=1" "SWH_DECODE_GRAPH_STEPS=16" "SWH_DECODE_L3_ATTN=64" "SWH_DECODE_L3_ATTN=128" "X=2" "SWH_DECODE_GRAPH_STEPS=32"; do
  r=$(env $v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$v $r" >> $o
  echo "$v $r"
done
