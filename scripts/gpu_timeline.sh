#!/bin/bash
# rocprofv3 kernel trace of a short bench run (BENCH_ARGS), reduced to the
# engine's kernels (name, start, end, queue/stream ids) in
# gpurun_out/$OUT_NAME/trace_small.csv for scripts/timeline*.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-tl}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- \
  python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 5} --no-cpu-baseline --no-parity > $O/b.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/b.log; exit $rc; }
f=$(find $O/p -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_reduce.py "$f" $O/trace_small.csv && rm -rf $O/p
