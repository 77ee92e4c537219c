#!/bin/bash
# Diagnostic: decide's per-DownTrack phases at the 10-ms tick (1,000 rooms),
# from the LKF_SVC_STATS build, with the kernel durations of the same run
# (rocprofv3 kernel trace) for the stats build and the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-tickst}; mkdir -p $O
for lib in liblkfwd_svcst.so; do
  LKF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${lib%.so} -o run -- \
    python3 -u scripts/svc_stats.py ${ST_ARGS:-1000 -1 2 0.01 0.2} > $O/stats_${lib%.so}.log 2>&1
  rc=$?; echo "$lib rc=$rc"; tail -3 $O/stats_${lib%.so}.log; [ $rc -eq 0 ] || exit $rc
  f=$(find $O/p_${lib%.so} -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/kstats_${lib%.so}.csv
  python3 - $O/kstats_${lib%.so}.csv <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print(f"  {r['Name'][:50]:50s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
done
exit 0
