#!/bin/bash
# Closing pass per bench shape (FINAL_SHAPES: '|'-separated "name:bench args"):
#   1. PMC passes, one rocprofv3 run per counter (FETCH_SIZE, WRITE_SIZE),
#      summarised per kernel (scripts/pmc_summary.py, tagged with the sources'
#      sha and the shape) and copied to profiles/${ROUND:-r5}_pmc_<name>.json so that
#   2. the bench line (with its CPU baseline) quotes the measured traffic,
#   3. rocprofv3 --kernel-trace --stats of the same command (kernel CSV).
# Outputs under gpurun_out/$OUT_NAME; every GPU step has its own limit and the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_NAME:-${ROUND:-r5}_final}
mkdir -p $O profiles
SHAPES="${FINAL_SHAPES:-c2:|c2ext:--extpackets}"
IFS='|' read -ra LIST <<< "$SHAPES"
for item in "${LIST[@]}"; do
  name=${item%%:*}
  args=${item#*:}
  if [ "${PMC:-1}" = "1" ]; then
    i=0
    CTRS="FETCH_SIZE WRITE_SIZE"
    # EXACT=1: the request counters by size as well (scripts/pmc_summary.py exact_bytes)
    [ "${EXACT:-1}" = "1" ] && CTRS="$CTRS TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum"
    for ctr in $CTRS; do
      timeout -k 10 300 rocprofv3 --pmc ${ctr//,/ } --kernel-trace --output-format csv -d $O/pmc_$name/p$i -o run -- \
        python3 bench.py $args --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_${name}_p$i.log 2>&1
      rc=$?; echo "$name pmc $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_${name}_p$i.log; exit $rc; }
      i=$((i+1))
    done
    BENCH_ARGS="$args" python3 scripts/pmc_summary.py $O/pmc_$name --delete-raw > $O/pmc_${name}_summary.log 2>&1 || exit 5
    cp $O/pmc_$name/summary.json profiles/${ROUND:-r5}_pmc_$name.json
    cp $O/pmc_$name/summary.json $O/${ROUND:-r5}_pmc_$name.json
    python3 -c "import json,sys; d=json.load(open('$O/${ROUND:-r5}_pmc_$name.json')); print('$name hbm_bytes_per_step', d.get('hbm_bytes_per_step'))"
  fi
  if [ "${BENCH:-1}" = "1" ]; then
    timeout -k 10 600 python3 bench.py $args --steps ${STEPS:-20} --warmup 5 ${BENCH_EXTRA:-} > $O/bench_$name.log 2>&1
    rc=$?; echo "$name bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$name.log; exit $rc; }
    grep '^{' $O/bench_$name.log | tail -1 > $O/bench_$name.json; cut -c1-300 $O/bench_$name.json
  fi
  if [ "${PROF:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
      python3 bench.py $args --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-parity > $O/prof_$name.log 2>&1
    rc=$?; echo "$name prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_$name.log; exit $rc; }
    f=$(find $O/prof_$name -name '*kernel_stats.csv' | head -1)
    [ -n "$f" ] && cp "$f" $O/kernel_stats_$name.csv
    find $O/prof_$name -name '*kernel_trace.csv' -delete
  fi
done
exit 0
