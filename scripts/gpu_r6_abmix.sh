#!/bin/bash
# (A/B) builds and environment settings on one bench shape, in one GPU call:
# MIX is a space-separated list of lib|ENV=value (ENV part may be empty).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT_NAME:-abmix}; mkdir -p $O
A=${MIX_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-parity}
for r in $(seq 1 ${MIX_REPS:-2}); do
  for cfg in ${MIX}; do
    lib=${cfg%%|*}; ev=${cfg#*|}
    env LKF_LIB=$lib $ev timeout -k 10 300 python3 bench.py $A > $O/run.log 2>&1 || { echo "$lib $ev failed"; tail -3 $O/run.log; exit 1; }
    python3 -c "
import json
d=[json.loads(l) for l in open('$O/run.log') if l.startswith('{')][-1]
print('%-18s %-18s ms=%.4f frac=%.4f' % ('$lib','$ev',d['ms_per_step'],d['roofline']['frac']))"
  done
done
