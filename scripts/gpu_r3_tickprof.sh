#!/bin/bash
# Kernel durations of the 10-ms tick at 1,000 rooms: pipelined and one batch
# at a time (--sync-each).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_tickprof}
mkdir -p $O
for mode in pipe sync; do
  extra=""; [ $mode = sync ] && extra="--sync-each"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$mode -o run -- python3 bench.py --batch-s 0.01 --rooms ${ROOMS:-1000} --steps 100 --warmup 20 --no-cpu-baseline $extra ${BENCH_ARGS:-} > $O/prof_$mode.log 2>&1
  rc=$?; echo "prof_$mode rc=$rc"; grep '^{' $O/prof_$mode.log | tail -1 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
  f=$(find $O/prof_$mode -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_$mode.csv && head -16 $O/kernel_stats_$mode.csv | cut -d, -f1-4
done
exit 0
