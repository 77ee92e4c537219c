#!/bin/bash
# Round-3 closing pass on one MI355X, from the tree as committed: the whole
# -m gpu suite, the headline bench (with its CPU baseline) and its rocprof
# kernel stats, every config's line, the deployment shapes (10-ms ticks,
# ingress, SRTP profiles), then the PMC passes for the traffic summary.
# Each GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_final}
mkdir -p $O
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -1 > $O/$name.json; cut -c1-200 $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
st bench_c2 300 python3 bench.py --steps 20 --warmup 5
st bench_c2_sync 300 python3 bench.py --steps 20 --warmup 5 --sync-each --no-cpu-baseline
for c in 1 3 4 5; do st bench_c$c 400 python3 bench.py --config $c --steps 10 --warmup 3; done
st tick100 240 python3 bench.py --batch-s 0.01 --steps 200 --warmup 20 --no-cpu-baseline
st tick1000 300 python3 bench.py --batch-s 0.01 --rooms 1000 --steps 200 --warmup 20 --no-cpu-baseline
st ingress 300 python3 bench.py --ingress --steps 10 --warmup 3 --no-cpu-baseline
st srtp_aes_cm 300 python3 bench.py --srtp --steps 10 --warmup 3 --no-cpu-baseline
st srtp_gcm 300 python3 bench.py --srtp --srtp-profile gcm --steps 10 --warmup 3 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.log 2>&1
echo "prof rc=$?"; f=$(find $O/prof_c2 -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_c2.csv && head -6 $O/kernel_stats_c2.csv | cut -d, -f1-4
PMC_NAME=${OUT_NAME:-r3_final}/pmc bash scripts/gpu_r3_pmc.sh
exit 0
