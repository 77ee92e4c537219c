set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/abside; mkdir -p $O
A='--steps 30 --warmup 5 --no-cpu-baseline --no-parity'
for r in 1 2; do
  for cfg in "liblkfwd.so|" "liblkfwd_n256.so|" "liblkfwd.so|LKF_SIDE_CUS=16" "liblkfwd.so|LKF_SIDE_CUS=24" "liblkfwd_n256.so|LKF_SIDE_CUS=24"; do
    lib=${cfg%%|*}; ev=${cfg#*|}
    env LKF_LIB=$lib $ev timeout -k 10 300 python3 bench.py $A > $O/run.log 2>&1 || { echo "$lib $ev failed"; tail -3 $O/run.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/run.log') if l.startswith('{')][-1]
print('%-18s %-16s ms=%.4f frac=%.4f' % ('$lib','$ev',d['ms_per_step'],d['roofline']['frac']))"
  done
done
