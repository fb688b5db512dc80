#!/bin/bash
# configs[3] 1/8-shard deterministic stream: A/B of tools/ab variants (AB="...") against the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in cur ${AB:-} cur; do
  lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
  WHARF_LIB_PATH=$lib timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --det --shard 8 --no-oracle > gpurun_out/c3det_ab_$v.log 2>&1 || exit 6
  echo "$v: $(grep -E '^batch' gpurun_out/c3det_ab_$v.log | sed 's/, affected.*//' | tr '\n' ' ')"
done
