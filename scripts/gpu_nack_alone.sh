#!/bin/bash
# k_ing_nack timed with the GPU to itself (LKF_NACK_ALONE=1: the rest of the
# ingest waits for it) on the headline shape, one batch at a time, for each
# library in NA_LIBS; the kernel stats go to gpurun_out/$OUT_NAME/<lib>_stats.csv.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-nack_alone}
mkdir -p $O
for lib in ${NA_LIBS:-liblkfwd.so}; do
  n=${lib%.so}
  LKF_NACK_ALONE=1 LKF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- \
    python3 bench.py ${NA_ARGS:-} --sync-each --steps 12 --warmup 4 --no-cpu-baseline --no-parity > $O/${n}.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/${n}.log; exit $rc; }
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/${n}_stats.csv
  f=$(find $O/$n -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && python3 scripts/trace_reduce.py "$f" $O/${n}_trace.csv
  rm -rf $O/$n
  python3 - "$O/${n}_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'nack' in x['Name'] or 'stream_wave' in x['Name']:
        print('   %-50s calls=%s avg_us=%.1f min_us=%.1f max_us=%.1f' % (x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e3, float(x['MinNs'])/1e3, float(x['MaxNs'])/1e3))
import os
t = sys.argv[1].replace('_stats.csv', '_trace.csv')
if os.path.exists(t):
    r = sorted(csv.DictReader(open(t)), key=lambda x: int(x['Start_Timestamp']))
    for x in r:
        if 'k_ing_nack' not in x['Kernel_Name']:
            continue
        s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
        ov = sorted(set(y['Kernel_Name'].split('(')[0][-24:] for y in r if y is not x and int(y['End_Timestamp']) > s and int(y['Start_Timestamp']) < e))
        print('     nack %.1f us; overlapping: %s' % ((e - s) / 1e3, ', '.join(ov)))
PY
done
exit 0
