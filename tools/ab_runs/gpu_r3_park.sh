#!/bin/bash
# node2vec re-walk by passes: parity of the re-walk paths, then configs[4] 1/8 shard (park vs sorted) at wpv 1 and 10.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3park; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "node2vec" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit $rc
for v in park sorted; do
  WHARF_N2V_REWALK=$v timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv1_$v.log 2>&1 || exit 6
  echo "wpv1 $v"; grep -E '^batch|^generate' $O/c4_wpv1_$v.log
done
WHARF_N2V_REWALK=park timeout -k 10 500 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_park.log 2>&1 || exit 8
echo "wpv10 park"; grep -E '^batch|^generate' $O/c4_wpv10_park.log
