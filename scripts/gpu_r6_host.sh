#!/bin/bash
# Round-6 host-side measurements: the host enqueue of the
# headline step broken down (LKF_HOST_PROF=1: Python queue_events / ingest /
# lkf_run, and lkf_run's own sections), and the host-fed deployment shape
# (--host-io: lkf_submit from pinned host memory + lkf_drain_run of the
# previous batch, PCIe both ways) with its breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-r6host}
mkdir -p $O
for sh in "hostprof:" "hostio:--host-io" "hostio_ingress:--host-io --config 3 --rooms 125"; do
  name=${sh%%:*}; args=${sh#*:}
  LKF_HOST_PROF=1 timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
  grep '^{' $O/$name.log | tail -1 > $O/$name.json
  grep -E "host ms|lkf host" $O/$name.log
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('  ms=%.4f value=%.4g parity=%s host_enqueue=%s host_io=%s' % (d['ms_per_step'], d['value'], d.get('parity'), d.get('host_enqueue_ms_per_step'), d.get('host_io')))"
done
exit 0
