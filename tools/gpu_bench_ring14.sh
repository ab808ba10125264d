set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r3_bench_ring14_ab.log
: > $o
for v in "X=1" "SWH_LM_RING14=1" "X=2" "SWH_LM_RING14=1" "X=3" "SWH_LM_RING14=1"; do
  r=$(env $v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$v $r" >> $o
  echo "$v $r"
done
