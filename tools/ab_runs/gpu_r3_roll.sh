#!/bin/bash
# Rolling half-chunk scan and copy (WHARF_SCAN_KERNEL=roll, WHARF_COPY_KERNEL=roll) vs the defaults: parity, then
# configs[2] det probe (scan-only and fused), alternated, with a kernel trace of each probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3roll; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or det" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
export TMPDIR=/tmp
for v in roll lean roll lean; do
  export WHARF_SCAN_KERNEL=$v
  if [ $v = roll ]; then export WHARF_COPY_KERNEL=roll; else export WHARF_COPY_KERNEL=chunked; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_rewalk_scan|k_rewalk_copy|k_rewalk_chunked|k_det_suffix" --output-format csv -d $O/tr_$v -o run -- python3 tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(grep -v '^[WEI]2026' $O/probedet_$v.log | tail -1)"
  grep -h "k_rewalk\|k_det" $O/tr_$v/run_kernel_stats.csv | cut -d, -f1-4
done
