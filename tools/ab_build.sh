#!/bin/bash
# Build A/B variants of libwharf_gpu.so into tools/ab/lib_<name>.so from the
# current sources with extra -D flags; run them with WHARF_LIB_PATH (gpu_check.sh ab).
#   tools/ab_build.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -e
cd "$(dirname "$0")/../dynamicgraphrepresentationlearning_amd/csrc"
mkdir -p ../../tools/ab
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  d=/tmp/wharf_ab_$name; mkdir -p $d
  for src in wharf_kernels wharf_api; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include $defs -c $src.hip -o $d/$src.o &
  done
  g++ -O2 -std=c++17 -fPIC -Wall -I../../include -c wharf_io.cpp -o $d/wharf_io.o
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_$name.so $d/wharf_kernels.o $d/wharf_api.o $d/wharf_io.o
  echo "built tools/ab/lib_$name.so ($defs)"
done
