#!/bin/bash
# Round-4 check: chosen GPU test files (PYTESTS, default the whole -m gpu
# suite), then bench lines + kernel stats (scripts/gpu_r4_prof.sh).  Each GPU
# step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r4_check}
mkdir -p $O
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest ${PYTESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
[ "${BENCH:-1}" = "1" ] || exit 0
OUT_NAME=${OUT_NAME:-r4_check} bash scripts/gpu_r4_prof.sh
