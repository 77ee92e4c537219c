#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_bisect
mkdir -p $O
for v in 5 1 2 3 4; do
  LKF_LIB=liblkfwd_svcab$v.so timeout -k 10 120 python3 scripts/debug_alloc_dd.py > $O/ab$v.log 2>&1
  rc=$?; echo "ab$v rc=$rc"; tail -12 $O/ab$v.log
  [ $rc -eq 0 ] || exit $rc
done
