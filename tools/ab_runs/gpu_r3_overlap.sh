#!/bin/bash
# Deterministic copy with overlap-ordered loads (WHARF_COPY_KERNEL=overlap; 5 waves default build, 4 waves in
# tools/ab/lib_ov4.so) vs the default copy: parity, then configs[2] det probe with kernel traces, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3overlap; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or rmat10 or edge_cases or batch_walk_update or det" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
export TMPDIR=/tmp
for v in ov5 ov4 base ov5 ov4 base; do
  unset WHARF_LIB_PATH
  case $v in ov5) export WHARF_COPY_KERNEL=overlap;; ov4) export WHARF_COPY_KERNEL=overlap WHARF_LIB_PATH=$PWD/tools/ab/lib_ov4.so;; base) export WHARF_COPY_KERNEL=chunked;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_rewalk_chunked|k_rewalk_copy|k_det_suffix" --output-format csv -d $O/tr_$v -o run -- python3 tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(grep -v '^[WEI]2026' $O/probedet_$v.log | tail -1 | cut -c1-110) | $(grep -h 'k_rewalk_chunked\|k_rewalk_copy' $O/tr_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)"
done
