#!/bin/bash
# Round-5 diagnostic call: the whole -m gpu suite on the product build (no -x:
# every failure listed), the DD-limit subset on the variant builds, the
# SVC-run stop counters (configs[4]), then A/Bs (stream-wave occupancy, prep
# CU reserve).  Each GPU step has its own limit; a crash or hang ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg1}; mkdir -p $O
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-480} python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -15
  [ $rc -le 1 ] || exit $rc
fi
K="${DBG_K:-provisional_pass_matches_oracle or dd_tracker_matches_oracle}"
for lib in ${DBG_LIBS:-liblkfwd.so liblkfwd_checked.so}; do
  LKF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_alloc_gpu.py tests/test_tracker_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "$K" > $O/$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; grep -E "PASS|FAIL|Error:|CK_|check" $O/$lib.log | head -20
  [ $rc -le 1 ] || exit $rc
done
if [ "${SVC:-1}" = "1" ]; then
  LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 500 > $O/svc_stats.log 2>&1
  rc=$?; echo "svc rc=$rc"; tail -12 $O/svc_stats.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${AB:-1}" = "1" ]; then
  AB_LIBS="liblkfwd.so liblkfwd_iw3.so liblkfwd_dw4.so" AB_REPS=2 \
  AB_SHAPES="--steps 20 --warmup 5 --no-cpu-baseline --no-parity|--batch-s 0.01 --rooms 1000 --steps 100 --warmup 20 --no-cpu-baseline --no-parity" \
  OUT_NAME=${OUT_NAME:-dbg1}/ab bash scripts/gpu_ab.sh || exit $?
  AB_LIBS="liblkfwd.so liblkfwd_w3.so" AB_REPS=2 AB_SHAPES="--config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity" \
  OUT_NAME=${OUT_NAME:-dbg1}/ab5 bash scripts/gpu_ab.sh || exit $?
  AB_ENVS="-|LKF_PREP_RESERVE=2|LKF_PREP_RESERVE=4|LKF_PREP_RESERVE=8" AB_REPS=1 \
  OUT_NAME=${OUT_NAME:-dbg1}/env bash scripts/gpu_env_ab.sh || exit $?
fi
exit 0
