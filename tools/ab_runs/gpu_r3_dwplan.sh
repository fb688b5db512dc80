#!/bin/bash
# DeepWalk MH re-walk: lock-step sweep vs plan scan + sorted re-walk (WHARF_DW_REWALK, an A/B switch since
# removed: the sweep won): parity, then
# configs[3] 1/8 shard (32 % of walks re-walk) and configs[2] (81 %), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3dwplan; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in plan sweep plan sweep; do
  export WHARF_DW_REWALK=$v
  timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --shard 8 --no-oracle > $O/c3_$v.log 2>&1 || exit 6
  echo "c3 $v: $(grep -E '^batch' $O/c3_$v.log | tr '\n' ' ' | cut -c1-500)"
done
for v in plan sweep plan sweep; do
  export WHARF_DW_REWALK=$v
  timeout -k 10 300 python tools/rewalk_probe.py --batches 4 > $O/c2_$v.log 2>&1 || exit 7
  echo "c2 $v: $(grep -v '^[WEI]2026' $O/c2_$v.log | tail -1 | cut -c1-200)"
done
