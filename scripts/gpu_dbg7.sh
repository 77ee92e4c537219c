#!/bin/bash
# Round-5 call: the -m gpu suite (product), the decide-priority A/B on the
# headline, and a kernel timeline of the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg7}; mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $O/pytest_gpu.log | cut -c1-1500 | tail -12
[ $rc -le 1 ] || exit $rc
AB_ENVS="-|LKF_DEC_PRIO=0" AB_REPS=2 OUT_NAME=${OUT_NAME:-dbg7}/env bash scripts/gpu_env_ab.sh || exit $?
OUT_NAME=${OUT_NAME:-dbg7}/tl bash scripts/gpu_timeline.sh || exit $?
exit 0
