set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mall_probe.py --attn-l3 > gpurun_out/r3_attn_l3b.log 2>&1 || { tail -20 gpurun_out/r3_attn_l3b.log; exit 1; }
grep "decode step" gpurun_out/r3_attn_l3b.log
