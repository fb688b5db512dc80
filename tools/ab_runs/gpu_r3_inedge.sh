#!/bin/bash
# Two-pass in-edge scan: parity (re-walk/update paths, stream tests), then configs[3] 1/8 shard (deterministic)
# and configs[4] 1/8 shard (node2vec wpv 10) batches, two-pass vs in place, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3inedge; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in two one two one; do
  if [ $v = one ]; then export WHARF_INEDGE_ONE_PASS=1; else unset WHARF_INEDGE_ONE_PASS; fi
  timeout -k 10 400 python tools/bigscale.py --scale 25 --samples 1200000000 --det --wpv 10 --shard 8 --batches 3 --no-oracle > $O/c3_det_$v.log 2>&1 || exit 6
  echo "c3 det $v: $(grep -E '^batch' $O/c3_det_$v.log | tr '\n' ' ' | cut -c1-400)"
done
for v in two one; do
  if [ $v = one ]; then export WHARF_INEDGE_ONE_PASS=1; else unset WHARF_INEDGE_ONE_PASS; fi
  timeout -k 10 500 python tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8 > $O/c4_$v.log 2>&1 || exit 7
  echo "c4 $v: $(grep -E '^batch' $O/c4_$v.log | tr '\n' ' ' | cut -c1-400)"
done
