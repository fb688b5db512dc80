#!/bin/bash
# Isolation run: the node2vec paths sorted/move-lazy (the combination of the faulted gsort/move test, without the
# global sort) and the block-staged re-walk, each test under a 60 s limit; then configs[2] node2vec A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3block; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths and node2vec and (move-lazy or block)" --timeout 60 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Timeout" $O/pt.log | tail -6; [ $rc -eq 0 ] || exit $rc
for v in sorted block sorted block; do
  WHARF_N2V_REWALK=$v timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > $O/c2n2v_$v.log 2>&1 || exit 6
  echo "c2 n2v $v: $(tail -1 $O/c2n2v_$v.log)"
done
