#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_split
mkdir -p $O
SPLITS=${SPLITS:-3700,3900,3990,4022,4029,4034,4035,4037} timeout -k 10 200 python3 scripts/debug_split.py > $O/split.log 2>&1
rc=$?; echo "rc=$rc"; cat $O/split.log | tail -40
