#!/bin/bash
# The whole -m gpu suite in one process (no -x: every failure is reported), then smoke().
# usage: bash tools/gpu_suite.sh <tag> [pytest -k expression]
set -u
mkdir -p gpurun_out
tag=${1:-suite}; shift || true
K=()
if [ $# -gt 0 ]; then K=(-k "$1"); fi
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread "${K[@]}" \
  > gpurun_out/${tag}_gpu_suite.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_gpu_suite.log | tail -30
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/${tag}_smoke.log
exit $rc
