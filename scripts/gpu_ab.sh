#!/bin/bash
# A/B timing of in-tree builds in one GPU call (AB_LIBS, default the product
# liblkfwd.so against lib/liblkfwd_ab.so from `make -C livekit-server_amd/csrc
# ab ABNAME=ab ABFLAGS=...`): every shape in AB_SHAPES ('|'-separated bench
# argument lists) runs each build in turn, AB_REPS rounds.  One line per run:
# build, shape, ms_per_step, value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-ab}
mkdir -p $O
SHAPES="${AB_SHAPES:---steps 30 --warmup 5 --no-cpu-baseline}"
IFS='|' read -ra LIST <<< "$SHAPES"
i=0
for a in "${LIST[@]}"; do
  for r in $(seq 1 ${AB_REPS:-2}); do
    for lib in ${AB_LIBS:-liblkfwd.so liblkfwd_ab.so}; do
      LKF_LIB=$lib timeout -k 10 300 python3 bench.py $a > $O/s${i}_${lib%.so}_$r.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || { echo "$lib shape$i rc=$rc"; tail -5 $O/s${i}_${lib%.so}_$r.log; exit $rc; }
      python3 - "$O/s${i}_${lib%.so}_$r.log" "$lib" "$a" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2]:16s} {sys.argv[3][:60]:60s} ms={d['ms_per_step']:.4f} value={d['value']:.4g} frac={d.get('roofline', {}).get('frac')}")
EOF
    done
  done
  i=$((i+1))
done
exit 0
