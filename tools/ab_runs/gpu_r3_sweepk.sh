#!/bin/bash
# DeepWalk sweep with K walks per lane (WHARF_SWEEP_WALKS=1/2/4, an A/B switch since removed: K=1 won): parity, then configs[3] 1/8 shard (32 % of
# walks re-walk) and configs[2] (81 %), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3sweepk; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in 2 1 4 2 1 4; do
  export WHARF_SWEEP_WALKS=$v
  timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --shard 8 --no-oracle > $O/c3_$v.log 2>&1 || exit 6
  echo "c3 K=$v: $(grep -E '^batch' $O/c3_$v.log | sed 's/, affected.*//' | tr '\n' ' ' | cut -c1-400)"
done
for v in 2 1 2 1; do
  export WHARF_SWEEP_WALKS=$v
  timeout -k 10 300 python tools/rewalk_probe.py --batches 4 > $O/c2_$v.log 2>&1 || exit 7
  echo "c2 K=$v: $(grep -v '^[WEI]2026' $O/c2_$v.log | tail -1 | cut -c1-200)"
done
