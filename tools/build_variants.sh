#!/bin/bash
# Build tuning/diagnostic variants of librsort in parallel:
#   tools/build_variants.sh name:-DA=1,-DB=2 [name2:...]  -> lib/variants/librsort_<name>.so
set -e
cd "$(dirname "$0")/../webgpu-radix-sort_amd/csrc"
mkdir -p ../lib/variants
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}; defs=${defs//,/ }
  echo "/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -fvisibility=hidden --offload-arch=gfx950 $defs -shared -o ../lib/variants/librsort_$name.so rsort.hip"
done | xargs -P 6 -I{} bash -c "{}"
