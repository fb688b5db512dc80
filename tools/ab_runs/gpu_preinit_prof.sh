#!/bin/bash
# Kernel trace of the configs[2] node2vec re-walk with and without the anchor pre-init.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pre lazy; do
  np=0; [ $v = lazy ] && np=1
  WHARF_NO_PREINIT=$np timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_preinit_$v -o run -- python3 tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/prof_preinit_$v.log 2>&1 || exit 6
done
for v in pre lazy; do echo $v; find gpurun_out/prof_preinit_$v -name "*kernel_stats.csv" -exec head -8 {} \; ; done
