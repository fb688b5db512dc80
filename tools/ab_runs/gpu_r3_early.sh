#!/bin/bash
# node2vec plan (and scan-only rewalk points) on a second stream beside the CSR update (WHARF_EARLY_PLAN=1,
# default) vs after it: the whole -m gpu suite, smoke, then the configs[2] node2vec probe and the configs[4]
# 1/8 shard (wpv 10), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3early; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 5
tail -1 $O/smoke.log
for i in 1 2; do for v in 1 0; do
  export WHARF_EARLY_PLAN=$v
  timeout -k 10 300 python3 tools/rewalk_probe.py --model node2vec --batches 4 > $O/probe_n2v_${v}_$i.log 2>&1 || exit 6
  echo "c2 n2v early=$v #$i: $(grep -v '^[WEI]20' $O/probe_n2v_${v}_$i.log | tail -1 | cut -c1-330)"
done; done
for v in 1 0; do
  export WHARF_EARLY_PLAN=$v
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_$v.log 2>&1 || exit 7
  echo "c4 wpv10 early=$v: $(grep -E '^batch' $O/c4_wpv10_$v.log | cut -c1-80 | tr '\n' ' ')"
done
