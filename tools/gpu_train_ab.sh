set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r3_train_ab.log
: > $o
for v in "X=1" "SWH_NORM_RPB=128" "SWH_DW_STREAM=0" "X=2" "SWH_NORM_RPB=64"; do
  echo "== $v" >> $o
  env $v timeout -k 10 240 python -u tools/train_kernels.py --reps 6 2>&1 | grep "half-step" >> $o || exit 1
done
cat $o
