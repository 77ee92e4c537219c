#!/bin/bash
# Round-5 call: the -m gpu suite twice (the intermittent DD-cursor failure),
# then the headline bench and its kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-dbg8}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu_$r.log 2>&1
  rc=$?; echo "pytest $r rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E  " $O/pytest_gpu_$r.log | cut -c1-600 | tail -8
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
OUT_NAME=${OUT_NAME:-dbg8}/tl bash scripts/gpu_timeline.sh || exit $?
exit 0
