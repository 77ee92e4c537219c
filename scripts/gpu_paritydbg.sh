#!/bin/bash
# Diagnostic: the ingress-inclusive parity gate as a function of the number
# of batches (warmup 5 + steps), with the gate's differing examples.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/paritydbg; mkdir -p $O
for k in ${PD_STEPS:-1 3 7 20}; do
  timeout -k 10 300 python3 bench.py --steps $k --warmup 5 --no-cpu-baseline ${PD_ARGS:-} > $O/steps$k.log 2>&1
  rc=$?; echo "steps $k rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/steps$k.log; exit $rc; }
  python3 - $O/steps$k.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
g = d.get("parity_gate") or {}
print(" parity", d.get("parity"), "dts_differing", g.get("downtracks_differing"), "counters", g.get("counters_gpu_oracle"))
for e in g.get("differing_examples", [])[:2]:
    print("  ", json.dumps(e)[:600])
PY
done
exit 0
