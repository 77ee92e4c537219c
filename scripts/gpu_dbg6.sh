#!/bin/bash
# Diagnostic: the allocation tests in order (the DD-cursor failure, with the
# allocations around it), the SVC-run counters + phase cycles (configs[4]),
# and a kernel timeline of the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg6}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_alloc_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "allocate_optimal or pause or provisional" > $O/alloc.log 2>&1
rc=$?; echo "alloc rc=$rc"; grep -E "PASSED|FAILED|^E  " $O/alloc.log | cut -c1-3000 | head -20
[ $rc -le 1 ] || exit $rc
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 500 > $O/svc_stats.log 2>&1
rc=$?; echo "svc rc=$rc"; tail -10 $O/svc_stats.log; [ $rc -eq 0 ] || exit $rc
OUT_NAME=${OUT_NAME:-dbg6}/tl bash scripts/gpu_timeline.sh || exit $?
exit 0
