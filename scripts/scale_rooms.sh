set -u
cd "${GRAFT_REPO_ROOT:-.}"
make -s -C oracle >/dev/null
for r in 12 25 50 100 200; do
  timeout -k 10 200 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --sync-each --rooms $r > gpurun_out/scale_$r.log 2>&1 || exit $?
  python3 - $r gpurun_out/scale_$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = {x["kernel"]: x["avg_ms"] for x in d["roofline"]["kernels"]}
print("rooms %4s fwd/step %9d decide %.4f emit %.4f" % (sys.argv[1], d["forwarded_per_step"], k["k_decide_dt"], k["k_emit"]))
PY
done
