set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_pmc.sh && bash tools/gpu_r3_v4.sh
