#!/bin/bash
# node2vec sorted re-walk with a wave's entries in column order (WHARF_N2V_LANE_SORT=1, default) vs list order:
# parity, configs[2] node2vec probe with kernel traces, configs[4] 1/8 shard, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3lanesort; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
export TMPDIR=/tmp
for v in 1 0 1 0; do
  export WHARF_N2V_LANE_SORT=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_rewalk_sorted|k_rewalk_plan" --output-format csv -d $O/n2v_$v -o run -- python3 tools/rewalk_probe.py --model node2vec --batches 3 > $O/proben2v_$v.log 2>&1 || exit 6
  echo "n2v sort=$v: $(grep -v '^[WEI]2026' $O/proben2v_$v.log | tail -1) | $(grep k_rewalk_sorted $O/n2v_$v/run_kernel_stats.csv | cut -d, -f3-4)"
done
for v in 1 0; do
  export WHARF_N2V_LANE_SORT=$v
  timeout -k 10 500 python tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8 > $O/c4_$v.log 2>&1 || exit 7
  echo "c4 sort=$v: $(grep -E '^batch' $O/c4_$v.log | tr '\n' ' ' | cut -c1-420)"
done
