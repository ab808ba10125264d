set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r3_graph_branch_probe.log
: > $o
timeout -k 10 120 python -u tools/graph_branch_probe.py >> $o 2>&1 || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python -u tools/graph_branch_probe.py >> $o 2>&1 || exit 1
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 120 python -u tools/graph_branch_probe.py >> $o 2>&1 || exit 1
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 120 python -u tools/graph_branch_probe.py >> $o 2>&1 || exit 1
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python -u tools/graph_branch_probe.py >> $o 2>&1 || exit 1
grep -v amdgpu.ids $o
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u tools/mall_probe.py --steps-only > gpurun_out/r3_mall_steps_nopc.log 2>&1 || exit 1
grep "decode step" gpurun_out/r3_mall_steps_nopc.log
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 300 python -u tools/mall_probe.py --steps-only > gpurun_out/r3_mall_steps_q2.log 2>&1 || exit 1
grep "decode step" gpurun_out/r3_mall_steps_q2.log
