#!/bin/bash
# The ingress-side checks after a bucket/TWCC change: RTX + ingress parity,
# then the raw-datagram bench lines (configs[1] --ingress and configs[2],
# whose speaker tick runs on the ingress path).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r3_ingress}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rtx_gpu.py tests/test_ingress_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
st() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -1 > $O/$name.json; cut -c1-300 $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
st bench_ingress 300 python3 bench.py --ingress --steps 10 --warmup 3
st bench_c3 400 python3 bench.py --config 3 --steps 10 --warmup 3
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ingress -o run -- python3 bench.py --ingress --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_ingress.log 2>&1
echo "prof rc=$?"; f=$(find $O/prof_ingress -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_ingress.csv && head -14 $O/kernel_stats_ingress.csv | cut -d, -f1-4
exit 0
