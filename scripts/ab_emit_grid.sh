set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for cfg in "0 24" "1 8" "1 12" "1 16" "1 24" "0 24"; do
  set -- $cfg
  LKF_EMIT_PERSISTENT=$1 LKF_EMIT_WG_PER_CU=$2 timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abe.log 2>&1 || { echo "fail $cfg"; tail -3 gpurun_out/abe.log; exit 1; }
  python3 - "$cfg" gpurun_out/abe.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = {x["kernel"]: x["avg_ms"] for x in d["roofline"]["kernels"]}
print("persist/wg %-6s value %.4g ms/step %.4f decide %.4f emit %.4f" % (sys.argv[1], d["value"], d["ms_per_step"], k["k_decide_dt"], k["k_emit"]))
PY
done
