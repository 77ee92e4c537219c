#!/bin/bash
# A/B of two in-tree builds (LKF_LIB names under livekit-server_amd/lib, A first):
# the parity suite on B, then the 10-ms tick at 1,000 rooms and the headline,
# alternating A/B twice.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_ab}
mkdir -p $O
A=${LIB_A:-liblkfwd_base.so}; B=${LIB_B:-liblkfwd.so}
timeout -k 10 400 env LKF_LIB=$B python -u -m pytest tests/test_parity_gpu.py tests/test_boundary_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in $A $B; do
    for shape in tick head; do
      args="--steps 20 --warmup 5"; [ $shape = tick ] && args="--batch-s 0.01 --rooms 1000 --steps 100 --warmup 20"
      timeout -k 10 240 env LKF_LIB=$L python3 bench.py $args --no-cpu-baseline > $O/${shape}_${L}_$r.log 2>&1
      rc=$?; printf "%s %s r%d rc=%d " $shape $L $r $rc
      python3 -c "import json; d=json.loads([l for l in open('$O/${shape}_${L}_$r.log') if l.startswith('{')][-1]); print(d['ms_per_step'], '%.4g' % d['value'], [(k['kernel'], k['avg_ms']) for k in d['roofline']['kernels']])"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
exit 0
