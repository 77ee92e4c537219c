#!/bin/bash
# One GPU pass on the tree as built here: the -m gpu suite (optionally a
# subset: PYTEST_ARGS), the headline bench, its rocprof kernel stats.  Each
# GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_run}
mkdir -p $O
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | tail -1 | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_PROF:-1}" = "1" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cp "$f" $O/kernel_stats.csv && head -12 $O/kernel_stats.csv | cut -d, -f1-4
  exit $rc
fi
