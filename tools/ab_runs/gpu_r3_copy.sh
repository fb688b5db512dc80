#!/bin/bash
# Deterministic suffix copy: parity of the re-walk paths, then A/B on configs[2] (deterministic probe, fused
# walk update per batch), alternated: lean at 5 and 4 waves, round-2 chunked copy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3copy; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or batch_walk_update or edge_cases or extreme or det" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in lean5 lean4 chunked lean5 lean4 chunked; do
  case $v in lean5) e="WHARF_COPY_KERNEL=lean WHARF_COPY_LEAN_WAVES=5";; lean4) e="WHARF_COPY_KERNEL=lean WHARF_COPY_LEAN_WAVES=4";; chunked) e="WHARF_COPY_KERNEL=chunked";; esac
  env $e timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(tail -1 $O/probedet_$v.log)"
done
timeout -k 10 400 python tools/bigscale.py --scale 25 --samples 1200000000 --det --wpv 10 --shard 8 --batches 3 --no-oracle > $O/c3_det_shard8.log 2>&1 || exit 7
grep -E "^batch|in-edge" $O/c3_det_shard8.log
