#!/bin/bash
# Round-6 closing pass, in parts (one GPU call each, PART=a|b|c|d):
#   a  the -m gpu suite, the same suite on the bounds-checked build, smoke(),
#      then configs[1] (headline, ingress) and its ExtPacket step
#   b  configs[0], configs[2], configs[3] (ingress and ExtPacket)
#   c  configs[4] (ingress and ExtPacket) and the 10-ms ticks
#   d  SRTP deployment shapes and the one-batch-at-a-time kernel stats
#   e  the host-side breakdown and the host-fed shape (scripts/gpu_r6_host.sh)
# Shapes go through scripts/gpu_final.sh (PMC traffic, bench line with its CPU
# baseline and parity gate, rocprofv3 kernel stats).  Every GPU step has its
# own time limit and the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export ROUND=r6
O=gpurun_out/r6_final
mkdir -p $O
case "${PART:-a}" in
a)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  LKF_LIB=liblkfwd_checked.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > $O/pytest_gpu_checked.log 2>&1
  rc=$?; echo "pytest checked rc=$rc"; tail -2 $O/pytest_gpu_checked.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
  OUT_NAME=r6_final FINAL_SHAPES="c2:|c2ext:--extpackets" bash scripts/gpu_final.sh
  ;;
b)
  OUT_NAME=r6_final FINAL_SHAPES="c1:--config 1|c3:--config 3|c4:--config 4|c4ext:--config 4 --extpackets" \
    bash scripts/gpu_final.sh
  ;;
c)
  OUT_NAME=r6_final FINAL_SHAPES="c5:--config 5|c5ext:--config 5 --extpackets|tick1000:--batch-s 0.01 --rooms 1000|tick1000ext:--batch-s 0.01 --rooms 1000 --extpackets|tick100ext:--batch-s 0.01 --extpackets" \
    bash scripts/gpu_final.sh
  ;;
d)
  for sh in "srtp_aes_cm:--extpackets --srtp" "srtp_gcm:--extpackets --srtp --srtp-profile gcm" "srtp_aes_cm_ingress:--srtp"; do
    name=${sh%%:*}; args=${sh#*:}
    timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$name.log 2>&1
    rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$name.log; exit $rc; }
    grep '^{' $O/bench_$name.log | tail -1 > $O/bench_$name.json; cut -c1-200 $O/bench_$name.json
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_srtp -o run -- \
    python3 bench.py --extpackets --srtp --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_srtp.log 2>&1
  rc=$?; echo "srtp prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $O/prof_srtp -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_srtp_aes_cm.csv
  find $O/prof_srtp -name '*kernel_trace.csv' -delete
  for sh in "c2_sync:--sync-each" "c2ext_sync:--extpackets --sync-each"; do
    name=${sh%%:*}; args=${sh#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
      python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/prof_$name.log 2>&1
    rc=$?; echo "$name prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
    f=$(find $O/prof_$name -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_$name.csv
    find $O/prof_$name -name '*kernel_trace.csv' -delete
  done
  ;;
e)
  OUT_NAME=r6_final bash scripts/gpu_r6_host.sh
  ;;
esac
exit 0
