#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3_svcdiag
mkdir -p $O
timeout -k 10 300 python3 scripts/svc_diag.py 200 3 > $O/dd.log 2>&1
rc=$?; echo "dd rc=$rc"; cat $O/dd.log
[ $rc -eq 0 ] || exit $rc
SVC_DD=0 timeout -k 10 300 python3 scripts/svc_diag.py 200 3 > $O/vp9.log 2>&1
rc=$?; echo "vp9 rc=$rc"; cat $O/vp9.log
exit $rc
