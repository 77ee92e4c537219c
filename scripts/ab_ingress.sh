#!/bin/bash
# A/B of engine library variants on the raw-datagram (ingress) bench:
#   LIBS="liblkfwd.so liblkfwd_x.so" bash scripts/ab_ingress.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS}; do
  LKF_LIB=livekit-server_amd/lib/$lib timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --ingress > gpurun_out/abi_$lib.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abi_$lib.log; exit 1; }
  python3 - "$lib" gpurun_out/abi_$lib.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-24s value %.4g  ms/step %.4f  gpu %.4f  host %.4f" % (sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["pipeline"]["gpu_ms_per_step"], d["host_enqueue_ms_per_step"]))
PY
done
