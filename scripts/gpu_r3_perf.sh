#!/bin/bash
# Round-3 measurement pass on one MI355X: store/load ceilings (micro), the
# headline bench standalone (--sync-each) and pipelined, every config's bench
# line, the headline's rocprof kernel stats and PMC passes.  Each GPU step has
# its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_perf}
mkdir -p $O
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -1 > $O/$name.json; tail -1 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
[ "${RUN_MICRO:-0}" = "1" ] && st micro 120 ./scripts/micro/fetch_calib 1024
st bench_c2 300 python3 bench.py --steps 20 --warmup 5
st bench_c2_sync 300 python3 bench.py --steps 20 --warmup 5 --sync-each --no-cpu-baseline
for c in 1 3 4 5; do st bench_c$c 400 python3 bench.py --config $c --steps 10 --warmup 3; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.log 2>&1
echo "prof rc=$?"
PMC_NAME=${OUT_NAME:-r3_perf}/pmc bash scripts/gpu_r3_pmc.sh
