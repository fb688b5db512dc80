#!/bin/bash
# Per-kernel VGPRs / occupancy of a HIP source (compile-time resource remarks).
#   tools/kernel_resources.sh <file.hip> [filter-regex] [extra hipcc flags...]
f=$1; pat=${2:-.}; shift 2 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$(dirname "$0")/../include" \
  -I"$(dirname "$0")/../dynamicgraphrepresentationlearning_amd/csrc" "$@" -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /ScratchSize/{sc=$5} /Occupancy/{print n, "vgpr="v, "scratch="sc, "waves/simd="$5}' |
  c++filt | grep -E "$pat"
