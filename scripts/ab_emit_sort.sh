#!/bin/bash
# A/B of the emit group order (LKF_EMIT_SORT=0/1): bench lines, a parity run
# with the sorted order, and PMC FETCH_SIZE / WRITE_SIZE of k_emit per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LKF_EMIT_SORT=1 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_parity_full_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1
rc=$?; echo "sorted-order parity rc=$rc"; tail -2 gpurun_out/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
VAR=LKF_EMIT_SORT VALS="0 1 0 1" BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash scripts/ab_env.sh || exit 3
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LKF_EMIT_SORT=$v timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_sort$v/$c -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sort${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; exit 4; }
  done
done
python3 - <<'PY'
import csv, glob
for v in (0, 1):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob("gpurun_out/pmc_sort%d/%s/**/*counter_collection.csv" % (v, c), recursive=True)
        vals = []
        for fn in f:
            for r in csv.DictReader(open(fn)):
                if "k_emit<" in r.get("Kernel_Name", "") and r.get("Counter_Name") == c:
                    vals.append(float(r["Counter_Value"]))
        print("sort=%d %s k_emit per launch (KB): %s" % (v, c, [round(x) for x in vals][-4:]))
PY
