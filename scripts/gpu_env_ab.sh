#!/bin/bash
# A/B of environment settings in one GPU call: every shape in AB_SHAPES
# ('|'-separated bench argument lists) runs under each setting in AB_ENVS
# ('|'-separated VAR=value lists, "-" for none), AB_REPS rounds.  One line per
# run: setting, shape, ms_per_step, value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-envab}
mkdir -p $O
IFS='|' read -ra SH <<< "${AB_SHAPES:---steps 20 --warmup 5 --no-cpu-baseline --no-parity}"
IFS='|' read -ra EN <<< "${AB_ENVS:--}"
i=0
for a in "${SH[@]}"; do
  for r in $(seq 1 ${AB_REPS:-2}); do
    j=0
    for ev in "${EN[@]}"; do
      [ "$ev" = "-" ] && ev=""
      env $ev timeout -k 10 300 python3 bench.py $a > $O/s${i}_e${j}_$r.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || { echo "env[$ev] shape$i rc=$rc"; tail -5 $O/s${i}_e${j}_$r.log; exit $rc; }
      python3 - "$O/s${i}_e${j}_$r.log" "$ev" "$a" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2] or 'default':28s} {sys.argv[3][:50]:50s} ms={d['ms_per_step']:.4f} value={d['value']:.4g} frac={d.get('roofline', {}).get('frac')}")
PY
      j=$((j+1))
    done
  done
  i=$((i+1))
done
exit 0
