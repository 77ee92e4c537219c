#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_wt5
mkdir -p $O
WT_CONFIG=5 timeout -k 10 200 python3 scripts/wave_timeline.py 400 2 > $O/wt5.log 2>&1
rc=$?; echo "rc=$rc"; cat $O/wt5.log | tail -40
