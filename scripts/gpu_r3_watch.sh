#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_watch
mkdir -p $O
LKF_LIB=liblkfwd_svcwatch.so timeout -k 10 120 python3 scripts/debug_alloc_dd.py > $O/watch.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "watch dt\|DD state" $O/watch.log | tail -80
