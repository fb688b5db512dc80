#!/bin/bash
# Split deterministic re-walk (scan + masked table writes) vs the fused copy: parity with the split forced, then configs[2] probe A/B + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WHARF_DET_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -m gpu -q -x \
  -k "det" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_detsplit.log 2>&1
rc=$?; tail -2 gpurun_out/pt_detsplit.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  WHARF_DET_SPLIT=$v timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > gpurun_out/probedet_split$v.log 2>&1 || exit 6
  echo "split=$v"; grep -E "^batch|median|fused" gpurun_out/probedet_split$v.log | tail -6
done
WHARF_DET_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_detsplit -o run -- python3 tools/rewalk_probe.py --det --batches 4 > gpurun_out/prof_detsplit.log 2>&1 || exit 7
find gpurun_out/prof_detsplit -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-150
