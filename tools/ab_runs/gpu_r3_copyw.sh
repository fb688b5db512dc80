#!/bin/bash
# Deterministic copy occupancy A/B on configs[2] (det probe, fused): 32-KiB filter at 5 waves (default), 16-KiB
# filter at the compiler's choice, 16-KiB filter forced to 6 waves (tools/ab/lib_copyw6.so), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3copyw; mkdir -p $O
for v in fb1 fb0 fb0w6 fb1 fb0 fb0w6; do
  unset WHARF_LIB_PATH WHARF_COPY_SMALL_BLOOM
  case $v in fb0) export WHARF_COPY_SMALL_BLOOM=1;; fb0w6) export WHARF_COPY_SMALL_BLOOM=1 WHARF_LIB_PATH=$PWD/tools/ab/lib_copyw6.so;; esac
  timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(tail -1 $O/probedet_$v.log)"
done
