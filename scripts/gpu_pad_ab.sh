set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_padding_gpu.py tests/test_rtx_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pad.log 2>&1
rc=$?; echo "pad pytest rc=$rc"; tail -8 gpurun_out/pytest_pad.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in liblkfwd_head.so liblkfwd.so liblkfwd_head.so liblkfwd.so; do
  LKF_LIB=livekit-server_amd/lib/$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$lib.log 2>&1 || exit 3
  grep '^{' gpurun_out/ab_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value']/1e9, d['ms_per_step'], [ (k['kernel'],k['avg_ms']) for k in d['roofline']['kernels']])"
done
