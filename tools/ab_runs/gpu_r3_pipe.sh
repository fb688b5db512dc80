#!/bin/bash
# Rewalk-point scan kernels: parity of the re-walk / scan paths, then A/B on configs[2] (deterministic
# probe; scan-only walk update per batch), alternated: first (default), big (round 2), pipe16, pipe32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3pipe3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or batch_walk_update or edge_cases or extreme" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in lean big first lean big first; do
  case $v in lean) e="WHARF_SCAN_KERNEL=lean";; first) e="WHARF_SCAN_KERNEL=first";; big) e="WHARF_SCAN_KERNEL=big";; pipe16) e="WHARF_SCAN_KERNEL=pipe WHARF_SCAN_SMALL_BLOOM=1";; esac
  env $e timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(tail -1 $O/probedet_$v.log)"
done
