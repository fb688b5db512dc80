#!/bin/bash
# Return-first inits on the configs[2] node2vec probe, alternated 3x (kernel trace of the re-walk kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3retfirst_c2; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do for v in 1 0; do
  export WHARF_RET_FIRST=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_rewalk_sorted|k_rewalk_plan|k_anchor_preinit" --output-format csv -d $O/n2v_${v}_$i -o run -- python3 tools/rewalk_probe.py --model node2vec --batches 4 > $O/probe_n2v_${v}_$i.log 2>&1 || exit 6
  echo "c2 n2v rf=$v #$i: $(grep -v '^[WEI]20' $O/probe_n2v_${v}_$i.log | tail -1 | cut -c1-200) | $(grep -h k_rewalk_sorted $O/n2v_${v}_$i/run_kernel_stats.csv | cut -d, -f3-5)"
done; done
