#!/bin/bash
# GPU-box check: build, parity tests, smoke, short bench.  Each GPU step has its
# own time limit; a crash/timeout (rc not in {0,1}) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
make -s -C oracle clean all > $OUT/build.log 2>&1 || { echo "oracle build failed"; exit 2; }
make -s -C livekit-server_amd/csrc >> $OUT/build.log 2>&1 || { echo "engine build failed"; exit 2; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} > $OUT/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -3 $OUT/bench.log
  exit $brc
fi
exit $rc
