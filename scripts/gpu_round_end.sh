#!/bin/bash
# Round-end check on one MI355X: the whole -m gpu suite, a host-side profile of
# lkf_run, then scripts/gpu_final.sh (PMC traffic, bench, rocprof per shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
LKF_HOST_PROF=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hostprof.log 2>&1 || exit 3
grep -i "host ms\|lkf_run host" gpurun_out/hostprof.log | tail -3
bash scripts/gpu_final.sh
