#!/bin/bash
# Build tuning/diagnostic variants of librsort in parallel:
#   tools/build_variants.sh name:-DA=1,-DB=2 [name2:...]  -> lib/variants/librsort_<name>.so
# (kernels + plans recompiled with the defines and -DRS_SWEEP=1, without which the library fixes every
# knob at its default; the multi-GPU group object linked as built)
set -e
cd "$(dirname "$0")/../webgpu-radix-sort_amd/csrc"
make -s ../build/rs_group.o
OUTD=${OUTD:-../lib/variants}; mkdir -p $OUTD
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}; defs=${defs//,/ }
  echo "/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -fvisibility=hidden --offload-arch=gfx950 -DRS_SWEEP=1 $defs -shared -o $OUTD/librsort_$name.so rsort.hip -Wl,$PWD/../build/rs_group.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
done | xargs -P 6 -I{} bash -c "{}"
