#!/bin/bash
# Early plan with 1 or 2 workgroups per CU (room for the CSR update's kernels) vs the plan after the update:
# configs[2] node2vec probe and configs[4] 1/8 shard (wpv 10), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3early2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paths" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for i in 1 2; do for v in e1 e2 off; do
  case $v in e1) export WHARF_EARLY_PLAN=1 WHARF_EARLY_PLAN_WGS=1;; e2) export WHARF_EARLY_PLAN=1 WHARF_EARLY_PLAN_WGS=2;; off) export WHARF_EARLY_PLAN=0;; esac
  timeout -k 10 300 python3 tools/rewalk_probe.py --model node2vec --batches 4 > $O/probe_n2v_${v}_$i.log 2>&1 || exit 6
  echo "c2 n2v $v #$i: $(grep -v '^[WEI]20' $O/probe_n2v_${v}_$i.log | tail -1 | cut -c80-200)"
done; done
for v in e1 off e1 off; do
  case $v in e1) export WHARF_EARLY_PLAN=1 WHARF_EARLY_PLAN_WGS=1;; off) export WHARF_EARLY_PLAN=0;; esac
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_$v.log 2>&1 || exit 7
  echo "c4 wpv10 $v: $(grep -E '^batch' $O/c4_wpv10_$v.log | cut -c1-70 | tr '\n' ' ')"
done
