#!/bin/bash
# Diagnostic: the DD cursors of every context across the allocation tests
# (LKF_DEBUG_DD=1), in test order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg5}; mkdir -p $O
LKF_DEBUG_DD=1 timeout -k 10 300 python -u -m pytest tests/test_alloc_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread -k "allocate_optimal or pause or provisional" > $O/alloc_dd.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|^E  " $O/alloc_dd.log | head -20
exit 0
