#!/bin/bash
# GPU-box: padding/RTX parity (or the whole -m gpu suite with FULL=1), then
# an A/B of bench.py between liblkfwd_head.so (a baseline build) and the
# current library.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_PAD:-0}" != 1 ]; then
  if [ "${FULL:-0}" = 1 ]; then T="tests"; else T="tests/test_padding_gpu.py tests/test_rtx_gpu.py"; fi
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pad.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_pad.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
[ -f livekit-server_amd/lib/liblkfwd_head.so ] || exit 0
for lib in liblkfwd_head.so liblkfwd.so liblkfwd_head.so liblkfwd.so; do
  LKF_LIB=livekit-server_amd/lib/$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$lib.log 2>&1 || exit 3
  grep '^{' gpurun_out/ab_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value']/1e9, d['ms_per_step'], [ (k['kernel'],k['avg_ms']) for k in d['roofline']['kernels']])"
done
