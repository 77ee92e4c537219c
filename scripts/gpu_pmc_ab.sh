#!/bin/bash
# Exact read/write bytes per kernel (request counters by size) for several
# in-tree builds (AB_LIBS) on one bench shape (AB_ARGS), plus one timed run of
# each: the A/B of a traffic change in one GPU call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-pmcab}
mkdir -p $O
ARGS="${AB_ARGS:-}"
for lib in ${AB_LIBS:-liblkfwd.so}; do
  n=${lib%.so}
  i=0
  for ctr in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    LKF_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$n/p$i -o run -- \
      python3 bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/${n}_p$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$n pmc rc=$rc"; tail -5 $O/${n}_p$i.log; exit $rc; }
    i=$((i+1))
  done
  BENCH_ARGS="$ARGS" python3 scripts/pmc_summary.py $O/$n --delete-raw > /dev/null 2>&1 || exit 5
  python3 - "$O/$n/summary.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = sorted([(k, v) for k, v in d.items() if k.endswith("_hbm_exact_rd_wr_per_launch")], key=lambda kv: -sum(kv[1]))
print(sys.argv[2], "step exact rd/wr MB: %.1f / %.1f" % (d.get("hbm_exact_read_per_step", 0) / 1e6, d.get("hbm_exact_write_per_step", 0) / 1e6))
for k, v in ks[:6]:
    print("   %-34s rd %7.1f  wr %7.1f MB" % (k.replace("_hbm_exact_rd_wr_per_launch", ""), v[0] / 1e6, v[1] / 1e6))
PY
  for r in 1 2; do
    LKF_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/${n}_b$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$n bench rc=$rc"; tail -5 $O/${n}_b$r.log; exit $rc; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/${n}_b$r.log') if l.startswith('{')][-1]); print('   bench ms=%.4f frac=%.4f emit_ms=%.4f dec_ms=%.4f' % (d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels'][1]['avg_ms'], d['roofline']['kernels'][0]['avg_ms']))"
  done
done
exit 0
