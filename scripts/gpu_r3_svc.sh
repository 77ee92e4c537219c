#!/bin/bash
# configs[4] (SVC + DD) with the SVC runs, and emit A/B variants on configs[1]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_svc}
mkdir -p $O
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
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
  python3 bench.py --config 5 --steps 3 --warmup 2 --no-cpu-baseline > $O/prof_c5.log 2>&1
rc=$?; echo "prof c5 rc=$rc"
exit $rc
