#!/bin/bash
# Round-3 fault investigation + baseline on one MI355X:
#  1. the GPU suite on the product build,
#  2. the GPU suite on the bounds-checked build (LKF_LIB=liblkfwd_checked.so:
#     every test ends with the checked kernels' violation record required empty),
#  3. the allocation tests under rocprofv3 --kernel-trace (dispatch order),
#  4. a short bench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_fault}
mkdir -p $O
PT="python -u -m pytest -p no:cacheprovider -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest product rc=$rc"; tail -3 $O/pytest_gpu.log
# rc 1 = test failures (read the log); anything else (timeout, crash) stops here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LKF_LIB=liblkfwd_checked.so timeout -k 10 600 $PT -x tests -m gpu > $O/pytest_gpu_checked.log 2>&1
rc=$?; echo "pytest checked rc=$rc"; tail -3 $O/pytest_gpu_checked.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_alloc -o run -- \
  python3 -m pytest -p no:cacheprovider -x -q tests/test_alloc_gpu.py > $O/trace_alloc.log 2>&1
rc=$?; echo "rocprof alloc rc=$rc"; tail -2 $O/trace_alloc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log
[ $rc -eq 0 ] || exit $rc
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (emit's access patterns)
if [ "${CALIB:-1}" = "1" ]; then
  timeout -k 10 120 ./scripts/micro/fetch_calib 1024 > $O/calib_time.log 2>&1
  rc=$?; echo "calib rc=$rc"; cat $O/calib_time.log
  [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/calib_$c -o run -- ./scripts/micro/fetch_calib 1024 > $O/calib_$c.log 2>&1
    rc=$?; echo "calib pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
