#!/bin/bash
# configs[4] 1/8 shard node2vec wpv 1: kernel traces of the re-walk variants (park / sorted / sorted without the sure-accept skip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3prof; mkdir -p $O
export TMPDIR=/tmp
for v in sorted park; do
  WHARF_N2V_REWALK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 tools/bigscale.py --model node2vec --wpv 1 --batches 2 --mixed --no-oracle --shard 8 > $O/c4_$v.log 2>&1 || exit 6
  echo "== $v"; grep -E '^batch' $O/c4_$v.log
done
WHARF_N2V_REWALK=sorted WHARF_NO_SURE_SKIP=1 timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 2 --mixed --no-oracle --shard 8 > $O/c4_sorted_nosure.log 2>&1 || exit 7
echo "== sorted, no sure-accept skip"; grep -E '^batch' $O/c4_sorted_nosure.log
find $O -name "*kernel_stats.csv" | head
