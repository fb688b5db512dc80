#!/bin/bash
# In-edge scan loads in flight per thread: paths parity, then configs[3] 1/8-shard det stream (in-edge scan ms) alternating tools/ab variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "paths or csr" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_inedge.log 2>&1
rc=$?; tail -2 gpurun_out/pt_inedge.log; [ $rc -eq 0 ] || exit $rc
for v in cur l1 l4 cur l1 l4; do
  lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
  WHARF_LIB_PATH=$lib timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --det --shard 8 --no-oracle > gpurun_out/inedge_c3_$v.log 2>&1 || exit 6
  echo "c3det $v: $(grep -E '^batch' gpurun_out/inedge_c3_$v.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ') | $(grep 'in-edge scan' gpurun_out/inedge_c3_$v.log | sed 's/.*in-edge scan/in-edge/')"
done
