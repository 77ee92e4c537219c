#!/bin/bash
# Round-end measurement of HEAD on one MI355X: bench (with the CPU baseline),
# rocprofv3 kernel stats, PMC FETCH_SIZE / WRITE_SIZE passes -> the traffic
# summary bench.py quotes, the bench again with that traffic, and the
# deployment-shape lines.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -1 > $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
step bench python3 bench.py --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 4; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc/$c -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 5; }
done
python3 scripts/pmc_summary.py $O/pmc --delete-raw > $O/pmc_summary.log 2>&1 || exit 6
cp $O/pmc/summary.json $O/pmc_traffic.json
LKF_PMC_CSV=$O/pmc_traffic.json step bench_traffic python3 bench.py --steps 20 --warmup 5
step tick10ms python3 bench.py --steps 300 --warmup 30 --batch-s 0.01 --no-cpu-baseline
T=400 step tick10ms_1000rooms python3 bench.py --steps 100 --warmup 10 --batch-s 0.01 --rooms 1000 --no-cpu-baseline
step tick100ms python3 bench.py --steps 100 --warmup 10 --batch-s 0.1 --no-cpu-baseline
step ingress python3 bench.py --steps 10 --warmup 2 --ingress --no-cpu-baseline
step srtp python3 bench.py --steps 10 --warmup 2 --srtp --no-cpu-baseline
step hostio python3 bench.py --steps 5 --warmup 2 --host-io --no-cpu-baseline
echo done
