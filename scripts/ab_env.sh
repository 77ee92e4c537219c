#!/bin/bash
# A/B of one environment variable over values: VAR=LKF_EMIT_WG_PER_CU VALS="8 16 32" bash scripts/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VALS}; do
  env ${VAR}=$v timeout -k 10 ${AB_TIMEOUT:-180} python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline} > gpurun_out/abenv_$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/abenv_$v.log; exit $rc; fi
  python3 - "$VAR=$v" gpurun_out/abenv_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = {x["kernel"]: x["avg_ms"] for x in d["roofline"]["kernels"]}
print("%-24s value %.4g  ms/step %.4f  decide %.4f  emit %.4f  gpu %.4f" % (sys.argv[1], d["value"], d["ms_per_step"], k.get("k_decide_dt", 0), k.get("k_emit", 0), d["roofline"]["pipeline"]["gpu_ms_per_step"]))
PY
done
