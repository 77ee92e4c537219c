#!/bin/bash
# Round-6 GPU step: selected GPU tests (R6_TESTS, pytest -k expression or file
# list), then bench shapes (R6_BENCH: '|'-separated argument lists).  Every GPU
# step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r6}
mkdir -p $O
if [ -n "${R6_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread $R6_TESTS ${R6_K:+-k "$R6_K"} > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${R6_BENCH:-}" ]; then
  IFS='|' read -ra LIST <<< "$R6_BENCH"
  i=0
  for a in "${LIST[@]}"; do
    timeout -k 10 ${BENCH_TIMEOUT:-400} python3 bench.py $a > $O/bench_$i.log 2>&1
    rc=$?; echo "bench $i rc=$rc: $a"
    [ $rc -eq 0 ] || { tail -8 $O/bench_$i.log; exit $rc; }
    grep '^{' $O/bench_$i.log | tail -1 > $O/bench_$i.json
    python3 -c "
import json; d=json.load(open('$O/bench_$i.json'))
print('  ms=%.4f value=%.4g frac=%s parity=%s coll=%s' % (d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('parity'), {k: d['collective'][k] for k in ('ticks','gather_ms_per_step','device_records_match_host')} if d.get('collective') else None))"
    i=$((i+1))
  done
fi
exit 0
