#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_svc4}
mkdir -p $O
PT="python -u -m pytest -p no:cacheprovider -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT -x tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest product rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
LKF_LIB=liblkfwd_checked.so timeout -k 10 300 $PT -x tests/test_parity_gpu.py tests/test_padding_gpu.py tests/test_alloc_gpu.py -m gpu > $O/pytest_checked.log 2>&1
rc=$?; echo "pytest checked rc=$rc"; tail -3 $O/pytest_checked.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/svc_diag.py 200 3 > $O/diag_dd.log 2>&1
rc=$?; echo "diag dd rc=$rc"; cat $O/diag_dd.log
[ $rc -eq 0 ] || exit $rc
WT_CONFIG=5 timeout -k 10 200 python3 scripts/wave_timeline.py 400 2 > $O/wt5.log 2>&1
rc=$?; echo "wt rc=$rc"; grep -v "waves alive" $O/wt5.log | head -16
[ $rc -eq 0 ] || exit $rc
run() {  # name, env, bench args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -c 300 $O/$name.json; echo
  return $rc
}
run c5 LKF_GRAPH=1 --config 5 --steps 5 --warmup 2 --no-cpu-baseline &&
run c5_sync LKF_GRAPH=1 --config 5 --steps 3 --warmup 2 --sync-each --no-cpu-baseline || exit $?
exit 0
