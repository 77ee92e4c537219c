#!/bin/bash
# Deployable-tick shapes on one MI355X: 10-ms batches at 100 and 1,000 rooms,
# with the per-wave DownTrack count swept (LKF_DECIDE_K, 0 = the engine's
# choice), plus the host-side profile of the 1,000-room tick.  Each GPU step
# has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_tick}
mkdir -p $O
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -1 > $O/$name.json; cut -c1-220 $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
st tick100 240 python3 bench.py --batch-s 0.01 --steps 200 --warmup 20 --no-cpu-baseline
for k in 0 8 16; do
  LKF_DECIDE_K=$k st tick1000_k$k 300 python3 bench.py --batch-s 0.01 --rooms 1000 --steps 200 --warmup 20 --no-cpu-baseline
done
LKF_HOST_PROF=1 st tick1000_hostprof 300 python3 bench.py --batch-s 0.01 --rooms 1000 --steps 200 --warmup 20 --no-cpu-baseline
grep "host ms" $O/tick1000_hostprof.log
# standalone kernel durations of the headline step (one batch at a time)
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sync -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-each > $O/prof_sync.log 2>&1
echo "prof_sync rc=$?"
f=$(find $O/prof_sync -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_sync.csv && head -6 $O/kernel_stats_sync.csv | cut -d, -f1-4
exit 0
