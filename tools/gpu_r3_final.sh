set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_r3_pmc.sh || exit 1
sed -e 's/r3_v2_/r3_v3_/g' tools/gpu_r3_v1.sh > /tmp/v3.sh && bash /tmp/v3.sh
