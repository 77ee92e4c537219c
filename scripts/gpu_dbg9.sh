#!/bin/bash
# Diagnostic: the SVC DownTracks' phase cycles (configs[4]), and the 10-ms
# tick at 1,000 rooms: bench, kernel stats and PMC traffic per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg9}; mkdir -p $O
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py 500 > $O/svc_stats.log 2>&1
rc=$?; echo "svc rc=$rc"; tail -12 $O/svc_stats.log; [ $rc -eq 0 ] || exit $rc
T="--batch-s 0.01 --rooms 1000"
timeout -k 10 300 python3 bench.py $T --steps 100 --warmup 20 --no-cpu-baseline --no-parity > $O/tick.log 2>&1
rc=$?; echo "tick rc=$rc"; tail -1 $O/tick.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ptick -o run -- python3 bench.py $T --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $O/ptick.log 2>&1
rc=$?; echo "tick prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/ptick -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/kernel_stats_tick.csv
PMC_NAME=${OUT_NAME:-dbg9}/pmc_tick BENCH_ARGS="$T --steps 20 --warmup 5 --no-cpu-baseline --no-parity" PMC_DELETE_RAW=1 bash scripts/gpu_pmc.sh || exit $?
exit 0
