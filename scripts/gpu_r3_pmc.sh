#!/bin/bash
# Per-kernel PMC passes of the headline bench (one counter group per rocprofv3
# run, --pmc only with --kernel-trace) + the available-counter list, then the
# summary (scripts/pmc_summary.py).  PMC_SETS overrides the groups ('|'
# separates passes); BENCH_ARGS the bench command line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_NAME:-r3_pmc}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
SETS="${PMC_SETS:-FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY}"
IFS='|' read -ra PASSES <<< "$SETS"
i=0
for set in "${PASSES[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
  i=$((i+1))
done
PMC_CONFIG=${PMC_CONFIG:-2} PMC_ROOMS=${PMC_ROOMS:-100} python3 scripts/pmc_summary.py $OUT --delete-raw > $OUT/summary.log 2>&1
echo "summary rc=$?"
exit 0
