#!/bin/bash
# Round 3: the whole -m gpu suite, smoke, then configs[4] 1/8 shard node2vec re-walk (park vs sorted, wpv 1 and 10).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/pt.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
tail -1 $O/smoke.log
for v in park sorted; do
  WHARF_N2V_REWALK=$v timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv1_$v.log 2>&1 || exit 6
  echo "wpv1 $v"; grep -E '^batch|^generate' $O/c4_wpv1_$v.log
done
timeout -k 10 500 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_park.log 2>&1 || exit 8
echo "wpv10 park"; grep -E '^batch|^generate' $O/c4_wpv10_park.log
