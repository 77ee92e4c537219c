#!/bin/bash
# Builds k_decide_dt A/B variants of the engine library (CPU-side, in-tree):
#   VARIANTS="o5:-DLKF_OOO_RUN=1 b5:-DLKF_OOO_RUN=0" bash scripts/build_ab.sh
# -> livekit-server_amd/lib/liblkfwd_<name>.so
set -eu
cd "$(dirname "$0")/../livekit-server_amd/csrc"
make -s
for v in ${VARIANTS}; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $flags -c forward_kernels.hip -o ../lib/fk_$name.o
  others=$(ls ../lib/*.o | grep -v -e '/forward_kernels.o$' -e '/fk_' -e '/synth')
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/liblkfwd_$name.so ../lib/fk_$name.o $others
  echo "built liblkfwd_$name.so ($flags)"
done
