#!/bin/bash
# PMC counter passes (each pass its own rocprofv3 run; --pmc only with
# --kernel-trace, never with sys/runtime/hip tracing).
# PMC_SETS="SQ_WAVES SQ_INSTS_VALU|FETCH_SIZE|WRITE_SIZE"  ('|' separates passes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_NAME:-pmc}
mkdir -p $OUT
IFS='|' read -ra SETS <<< "${PMC_SETS:-FETCH_SIZE|WRITE_SIZE}"
i=0
for set in "${SETS[@]}"; do
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
  i=$((i+1))
done
python3 scripts/pmc_summary.py $OUT ${PMC_DELETE_RAW:+--delete-raw} > $OUT/summary.log 2>&1
exit 0
