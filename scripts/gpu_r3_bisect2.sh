#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_bisect2
mkdir -p $O
LKF_LIB=liblkfwd.so timeout -k 10 120 python3 scripts/debug_alloc_dd.py > $O/main.log 2>&1
rc=$?; echo "rc=$rc"; tail -40 $O/main.log
