#!/bin/bash
# Round-6 diagnosis: NACK/bench-shape tests, a kernel-trace timeline of the
# default bench (gpurun_out/$OUT_NAME/trace_small.csv) and the one-batch-at-a-time
# kernel stats (--sync-each).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r6diag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ingress_gpu.py tests/test_bench_shape_gpu.py -k "nack or bench_shape or config2" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- \
  python3 bench.py ${BENCH_ARGS:-} --steps 12 --warmup 4 --no-cpu-baseline --no-parity > $O/tl.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/tl.log; exit $rc; }
f=$(find $O/tl -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_reduce.py "$f" $O/trace_small.csv && rm -rf $O/tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sync -o run -- \
  python3 bench.py ${BENCH_ARGS:-} --sync-each --steps 12 --warmup 4 --no-cpu-baseline --no-parity > $O/sync.log 2>&1
rc=$?; echo "sync stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/sync.log; exit $rc; }
f=$(find $O/sync -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_sync.csv
rm -rf $O/sync
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-400
exit 0
