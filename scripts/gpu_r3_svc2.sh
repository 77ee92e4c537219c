#!/bin/bash
# SVC parity (config-5 GPU tests on the product and checked builds), then configs[4] bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_svc2}
mkdir -p $O
PT="python -u -m pytest -p no:cacheprovider -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT -x tests/test_parity_gpu.py tests/test_boundary_gpu.py -m gpu > $O/pytest_svc.log 2>&1
rc=$?; echo "pytest product rc=$rc"; tail -3 $O/pytest_svc.log
[ $rc -eq 0 ] || exit $rc
LKF_LIB=liblkfwd_checked.so timeout -k 10 300 $PT -x tests/test_parity_gpu.py -m gpu -k "config5" > $O/pytest_svc_checked.log 2>&1
rc=$?; echo "pytest checked rc=$rc"; tail -3 $O/pytest_svc_checked.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env, bench args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -c 300 $O/$name.json; echo
  return $rc
}
run c5 LKF_GRAPH=1 --config 5 --steps 5 --warmup 2 --no-cpu-baseline &&
run c5_sync LKF_GRAPH=1 --config 5 --steps 3 --warmup 2 --sync-each --no-cpu-baseline || exit $?
for v in liblkfwd.so liblkfwd_xcd0.so liblkfwd_nt0.so liblkfwd_nt0xcd0.so; do
  run ab_$v LKF_LIB=$v --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  run ab_sync_$v LKF_LIB=$v --steps 10 --warmup 3 --sync-each --no-cpu-baseline || exit $?
done
exit 0
