#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here;
# counters go in their own pass: scripts/gpu_pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_NAME:-prof}
mkdir -p $OUT
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu-baseline} > $OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 $OUT/bench.log
find $OUT -name "*kernel_stats.csv" | head -3
exit $rc
