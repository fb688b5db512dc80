#!/bin/bash
# Deterministic copy settling positives by the source index (default) vs bitmap word then index: parity, then
# configs[2] det probe with kernel traces, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3copyidx; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or det" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
export TMPDIR=/tmp
for v in 0 1 0 1; do
  export WHARF_COPY_BITMAP=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_rewalk_chunked|k_det_suffix" --output-format csv -d $O/tr_$v -o run -- python3 tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det bitmap=$v: $(grep -v '^[WEI]2026' $O/probedet_$v.log | tail -1) | $(grep k_rewalk_chunked $O/tr_$v/run_kernel_stats.csv | cut -d, -f3-4)"
done
