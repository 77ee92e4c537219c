#!/bin/bash
# GPU check of a decide change: the GPU test suite, the SVC phase cycles
# (LKF_SVC_STATS build), then an A/B of configs[4] and the headline against
# AB_OTHER (default liblkfwd_nofb.so).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r5b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ "${R5B_SVC:-1}" = 1 ]; then
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 500 > $O/svc_stats.log 2>&1
rc=$?; echo "svc rc=$rc"; tail -12 $O/svc_stats.log; [ $rc -eq 0 ] || exit $rc
fi
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 1000 -1 2 0.01 0.2 > $O/tick_stats.log 2>&1
rc=$?; echo "tick stats rc=$rc"; tail -4 $O/tick_stats.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --batch-s 0.01 --rooms 1000 --steps 100 --warmup 20 --no-cpu-baseline --no-parity > $O/tick.log 2>&1
rc=$?; echo "tick rc=$rc"; tail -1 $O/tick.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
OUT_NAME=${OUT_NAME:-r5b}/ab AB_LIBS="liblkfwd.so ${AB_OTHER:-liblkfwd_nofb.so}" AB_REPS=2 \
  AB_SHAPES="${R5B_SHAPES:---config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-parity|--steps 30 --warmup 5 --no-cpu-baseline --no-parity}" \
  bash scripts/gpu_ab.sh
