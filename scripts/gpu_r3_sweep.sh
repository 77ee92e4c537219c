#!/bin/bash
# Headline bench under engine knobs (env assignments in SWEEP, ';'-separated,
# "-" = defaults).  Each GPU step has its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_sweep}
mkdir -p $O
IFS=';' read -ra CASES <<< "${SWEEP:--}"
i=0
for c in "${CASES[@]}"; do
  i=$((i+1))
  envs=""; [ "$c" != "-" ] && envs="$c"
  timeout -k 10 240 env $envs python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/case$i.log 2>&1
  rc=$?; printf "case%d [%s] rc=%d " $i "$c" $rc; grep '^{' $O/case$i.log | tail -1 > $O/case$i.json
  python3 -c "import json; d=json.load(open('$O/case$i.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], [(k['kernel'], k['avg_ms']) for k in d['roofline']['kernels']])"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
