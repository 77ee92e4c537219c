#!/bin/bash
# Diagnostic: SVC/DD decide phase cycles on configs[4] (LKF_SVC_STATS build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-svcst}; mkdir -p $O
LKF_LIB=liblkfwd_svcst.so timeout -k 10 300 python3 -u scripts/svc_stats.py ${ST_ARGS:-500} > $O/svc_stats.log 2>&1
rc=$?; echo "svc rc=$rc"; tail -14 $O/svc_stats.log; exit $rc
