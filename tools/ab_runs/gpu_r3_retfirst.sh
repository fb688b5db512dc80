#!/bin/bash
# Return-first node2vec WEIGHT inits (WHARF_RET_FIRST=1, default) vs the full init on every uncached anchor:
# parity, configs[4] 1/8 shard (wpv 10 and 1) and the configs[2] node2vec probe, alternated on one box;
# (run 1 also tried the N>1 bench path over RCCL with 2 ranks on the one GPU: RCCL refuses, duplicate GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3retfirst${RF_RUN:-}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or node2vec or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in 1 0 1 0; do
  export WHARF_RET_FIRST=$v
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10_$v.log 2>&1 || exit 7
  echo "c4 wpv10 rf=$v: $(grep -E '^batch' $O/c4_wpv10_$v.log | cut -c1-150 | tr '\n' ' ')"
done
for v in 1 0; do
  export WHARF_RET_FIRST=$v
  timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv1_$v.log 2>&1 || exit 8
  echo "c4 wpv1 rf=$v: $(grep -E '^batch' $O/c4_wpv1_$v.log | cut -c1-150 | tr '\n' ' ')"
done
for v in 1 0; do
  export WHARF_RET_FIRST=$v
  timeout -k 10 300 python3 tools/rewalk_probe.py --model node2vec --batches 4 > $O/probe_n2v_$v.log 2>&1 || exit 9
  echo "c2 n2v rf=$v: $(grep -v '^[WEI]20' $O/probe_n2v_$v.log | tail -1 | cut -c1-300)"
done
