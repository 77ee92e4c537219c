#!/bin/bash
# Round-5 GPU call: the -m gpu suite (PYTEST=0 skips it; PYTEST_K selects),
# then an A/B of in-tree builds over bench shapes (scripts/gpu_ab.sh; AB=0
# skips it).  Each GPU step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r5}
mkdir -p $O
if [ "${PYTEST:-1}" = "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${AB:-1}" = "1" ]; then
  OUT_NAME=${OUT_NAME:-r5}/ab bash scripts/gpu_ab.sh || exit $?
fi
exit 0
