#!/bin/bash
# In-edge scan with the next group's loads issued before the positives are settled (WHARF_INEDGE_PREFETCH=1,
# 4 or 2 loads per group) vs without: parity, then configs[3] det and configs[4] node2vec 1/8-shard batches
# (graph update incl. the in-edge scan), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3inedge_pf; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in ie_pf0 ie_pf1 ie_pf1l2 ie_pf0 ie_pf1 ie_pf1l2; do
  export WHARF_LIB_PATH=$PWD/tools/ab/lib_$v.so
  timeout -k 10 400 python tools/bigscale.py --scale 25 --samples 1200000000 --det --wpv 10 --shard 8 --batches 3 --no-oracle > $O/c3_det_$v.log 2>&1 || exit 6
  echo "c3 det $v: $(grep -E '^batch' $O/c3_det_$v.log | cut -c1-60 | tr '\n' ' ')"
done
for v in ie_pf0 ie_pf1 ie_pf1l2; do
  export WHARF_LIB_PATH=$PWD/tools/ab/lib_$v.so
  timeout -k 10 500 python tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8 > $O/c4_$v.log 2>&1 || exit 7
  echo "c4 $v: $(grep -E '^batch' $O/c4_$v.log | cut -c1-60 | tr '\n' ' ')"
done
