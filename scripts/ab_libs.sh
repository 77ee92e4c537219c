#!/bin/bash
# A/B of engine library builds (livekit-server_amd/lib/<name>), optionally
# after a parity run of the default build:
#   PARITY="tests/test_parity_gpu.py" LIBS="liblkfwd_x.so liblkfwd.so" bash scripts/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PARITY:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PARITY -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_parity.log 2>&1
  rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/ab_parity.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for lib in ${LIBS}; do
    LKF_LIB=livekit-server_amd/lib/$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$lib.log 2>&1 || exit 3
    grep '^{' gpurun_out/ab_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']/1e9,4), d['ms_per_step'], [(k['kernel'],k['avg_ms']) for k in d['roofline']['kernels']], d['roofline']['pipeline']['gpu_ms_per_step'])"
  done
done
