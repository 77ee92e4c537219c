#!/bin/bash
# SRTP protect on one MI355X: the parity tests, then the --srtp bench line and
# its rocprof kernel stats for each profile.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_srtp}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_srtp_gpu.py ${PYTEST_EXTRA:-} -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for p in aes_cm gcm; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$p -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --srtp --srtp-profile $p > $O/bench_$p.log 2>&1
  rc=$?; echo "bench_$p rc=$rc"; grep '^{' $O/bench_$p.log | tail -1 > $O/bench_$p.json; python3 -c "import json,sys; d=json.load(open('$O/bench_$p.json')); print(d['ms_per_step'], d['srtp'])"
  [ $rc -eq 0 ] || exit $rc
  f=$(find $O/prof_$p -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_$p.csv && grep srtp_protect $O/kernel_stats_$p.csv | cut -d, -f1-4
done
exit 0
