set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_kmajor.sh && bash tools/gpu_sq_pmc.sh
