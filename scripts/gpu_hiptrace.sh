#!/bin/bash
# Diagnostic: the host side of the 10-ms tick (1,000 rooms) — HIP API calls
# per step and their host time (rocprofv3 HIP runtime trace, no counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-hiptrace}; mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d $O/p -o run -- \
  python3 bench.py --batch-s 0.01 --rooms 1000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $O/bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $O/bench.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
for f in $(find $O/p -name '*_stats.csv'); do cp $f $O/; done
ls $O
exit 0
