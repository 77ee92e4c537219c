#!/bin/bash
# Bench lines + rocprofv3 kernel stats of chosen bench shapes (round 4).
# PROF_SHAPES: '|'-separated bench argument lists (default: the ingress-inclusive
# headline step and the ExtPacket step).  OUT_NAME names the output
# directory under gpurun_out/.  Each GPU step has its own limit; the script
# stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r4_prof}
mkdir -p $O
SHAPES="${PROF_SHAPES:---steps 20 --warmup 5 --no-cpu-baseline|--extpackets --steps 20 --warmup 5 --no-cpu-baseline}"
IFS='|' read -ra LIST <<< "$SHAPES"
if [ "${RUN_TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in "${LIST[@]}"; do
  timeout -k 10 300 python3 bench.py $a > $O/bench$i.log 2>&1
  rc=$?; echo "bench$i ($a) rc=$rc"; grep '^{' $O/bench$i.log | tail -1 > $O/bench$i.json; cut -c1-400 $O/bench$i.json
  [ $rc -eq 0 ] || { tail -5 $O/bench$i.log; exit $rc; }
  if [ "${PROF:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$i -o run -- python3 bench.py $a > $O/prof$i.log 2>&1
    rc=$?; echo "prof$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof$i.log; exit $rc; }
    f=$(find $O/prof$i -name '*kernel_stats.csv' | head -1)
    [ -n "$f" ] && cp "$f" $O/kernel_stats$i.csv && head -20 $O/kernel_stats$i.csv | cut -d, -f1-5
    f=$(find $O/prof$i -name "*kernel_trace.csv" -size -20M | head -1); [ -n "$f" ] && cp "$f" $O/kernel_trace$i.csv
    find $O/prof$i -name "*kernel_trace.csv" -delete
  fi
  i=$((i+1))
done
exit 0
