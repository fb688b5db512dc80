#!/bin/bash
# Anchor carry (node2vec MH, undirected graphs: the sources' row entries travel through the merge, the
# ones a changed edge can affect are reset; WHARF_ANCHOR_CARRY=1, default) vs every entry of a rebuilt row
# reset: the whole -m gpu suite, then configs[4] 1/8 shard (wpv 10 and 1) and the configs[2] node2vec probe,
# alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3carry${CARRY_RUN:-}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in 1 0 1 0; do
  export WHARF_ANCHOR_CARRY=$v
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_$v.log 2>&1 || exit 7
  echo "c4 wpv10 carry=$v: $(grep -E '^batch' $O/c4_wpv10_$v.log | cut -c1-150 | tr '\n' ' ')"
done
for v in 1 0; do
  export WHARF_ANCHOR_CARRY=$v
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv1_$v.log 2>&1 || exit 8
  echo "c4 wpv1 carry=$v: $(grep -E '^batch' $O/c4_wpv1_$v.log | cut -c1-150 | tr '\n' ' ')"
done
for v in 1 0 1 0; do
  export WHARF_ANCHOR_CARRY=$v
  timeout -k 10 300 python3 tools/rewalk_probe.py --model node2vec --batches 4 > $O/probe_n2v_$v.log 2>&1 || exit 9
  echo "c2 n2v carry=$v: $(grep -v '^[WEI]20' $O/probe_n2v_$v.log | tail -1 | cut -c1-330)"
done
