#!/bin/bash
# Round-5 call: the -m gpu suite on the product build, the SVC-run stop
# counters (configs[4]), then A/Bs on configs[4] (in-run chain events, the DD
# decide occupancy) and the headline (decide occupancy).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg3}; mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 500 > $O/svc_stats.log 2>&1
rc=$?; echo "svc rc=$rc"; tail -8 $O/svc_stats.log; [ $rc -eq 0 ] || exit $rc
AB_LIBS="liblkfwd.so liblkfwd_noch.so liblkfwd_w3.so" AB_REPS=2 AB_SHAPES="--config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity" \
  OUT_NAME=${OUT_NAME:-dbg3}/ab5 bash scripts/gpu_ab.sh || exit $?
AB_LIBS="liblkfwd.so liblkfwd_dw4.so" AB_REPS=2 AB_SHAPES="--steps 20 --warmup 5 --no-cpu-baseline --no-parity" \
  OUT_NAME=${OUT_NAME:-dbg3}/ab bash scripts/gpu_ab.sh || exit $?
exit 0
