#!/bin/bash
# The re-walk / scan paths' parity, then A/B of the streaming kernels' filters on configs[2] (deterministic probe:
# scan-only + suffix copy per batch), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3stream; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or edge_cases or extreme" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in big small big small; do
  sm=0; [ $v = small ] && sm=1
  WHARF_SCAN_SMALL_BLOOM=$sm WHARF_COPY_SMALL_BLOOM=$sm timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(tail -1 $O/probedet_$v.log)"
done
