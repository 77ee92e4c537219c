#!/bin/bash
# Graph-replayed prep/scan stages: GPU suite (product + bounds-checked builds),
# then the 1-s headline and the 10-ms deployable tick at 100 and 1000 rooms,
# each with LKF_GRAPH=1 (default) and LKF_GRAPH=0 (direct launches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_graph}
mkdir -p $O
PT="python -u -m pytest -p no:cacheprovider -v --timeout 120 --timeout-method thread"
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 $PT -x tests -m gpu > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest product rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  LKF_LIB=liblkfwd_checked.so timeout -k 10 600 $PT -x tests -m gpu > $O/pytest_gpu_checked.log 2>&1
  rc=$?; echo "pytest checked rc=$rc"; tail -3 $O/pytest_gpu_checked.log
  [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, env, bench args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -c 400 $O/$name.json; echo
  return $rc
}
run c2_g1 LKF_GRAPH=1 --steps 20 --warmup 5 --no-cpu-baseline &&
run c2_g0 LKF_GRAPH=0 --steps 20 --warmup 5 --no-cpu-baseline &&
run tick100_g1 LKF_GRAPH=1 --steps 300 --warmup 30 --batch-s 0.01 --no-cpu-baseline &&
run tick100_g0 LKF_GRAPH=0 --steps 300 --warmup 30 --batch-s 0.01 --no-cpu-baseline &&
run tick1000_g1 LKF_GRAPH=1 --steps 200 --warmup 20 --batch-s 0.01 --rooms 1000 --no-cpu-baseline &&
run tick1000_g0 LKF_GRAPH=0 --steps 200 --warmup 20 --batch-s 0.01 --rooms 1000 --no-cpu-baseline &&
run s1000_g1 LKF_GRAPH=1 --steps 10 --warmup 3 --rooms 1000 --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tick100 -o run -- \
  python3 bench.py --steps 100 --warmup 10 --batch-s 0.01 --no-cpu-baseline > $O/prof_tick100.log 2>&1
rc=$?; echo "prof tick rc=$rc"
[ $rc -eq 0 ] || exit $rc
run c5_sync LKF_GRAPH=1 --config 5 --steps 3 --warmup 2 --sync-each --no-cpu-baseline || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
  python3 bench.py --config 5 --steps 3 --warmup 2 --no-cpu-baseline > $O/prof_c5.log 2>&1
rc=$?; echo "prof c5 rc=$rc"
exit $rc
