#!/bin/bash
# Copies the round-5 closing pass (gpurun_out/r5_final) into profiles/.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r5_final
for f in $O/bench_*.json; do [ -f "$f" ] && cp "$f" profiles/r5_final_$(basename $f); done
for f in $O/kernel_stats_*.csv; do [ -f "$f" ] && cp "$f" profiles/r5_final_$(basename $f); done
for f in $O/r5_pmc_*.json; do [ -f "$f" ] && cp "$f" profiles/$(basename $f); done
for f in pytest_gpu pytest_gpu_checked smoke; do [ -f $O/$f.log ] && cp $O/$f.log profiles/r5_final_$f.log; done
ls profiles | grep '^r5_' | wc -l
