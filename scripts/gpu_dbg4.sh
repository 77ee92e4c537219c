#!/bin/bash
# Round-5 call: the -m gpu suite on the product build and on the bounds-checked
# build (every failure listed, no -x), then configs[4]'s kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg4}; mkdir -p $O
for lib in liblkfwd.so liblkfwd_checked.so; do
  LKF_LIB=$lib timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_$lib.log 2>&1
  rc=$?; echo "$lib pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $O/pytest_$lib.log | tail -12
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run -- python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $O/prof5.log 2>&1
rc=$?; echo "prof5 rc=$rc"; tail -1 $O/prof5.log | cut -c1-200
f=$(find $O/prof5 -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/kernel_stats_c5.csv
exit 0
