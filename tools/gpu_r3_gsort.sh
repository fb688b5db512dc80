#!/bin/bash
# node2vec re-walk list sorted per block (0) vs globally by rewalk point (1): parity paths, configs[4] shard wpv 10 / 1, configs[2]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3gsort; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "paths and node2vec" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || exit $rc
for gs in 0 1 0 1; do
  WHARF_N2V_GLOBAL_SORT=$gs timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8 > $O/c4w10_gs$gs.log 2>&1 || exit 6
  echo "c4 wpv10 gs=$gs: $(grep -E '^batch' $O/c4w10_gs$gs.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
done
for gs in 0 1; do
  WHARF_N2V_GLOBAL_SORT=$gs timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 2 --mixed --no-oracle --shard 8 > $O/c4w1_gs$gs.log 2>&1 || exit 7
  echo "c4 wpv1 gs=$gs: $(grep -E '^batch' $O/c4w1_gs$gs.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
  WHARF_N2V_GLOBAL_SORT=$gs timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > $O/c2n2v_gs$gs.log 2>&1 || exit 8
  echo "c2 n2v gs=$gs: $(tail -1 $O/c2n2v_gs$gs.log)"
done
