#!/bin/bash
# Round 3 baseline: configs[4] 1/8-shard node2vec mixed batches at wpv 1 and wpv 10 (HEAD), init counters at wpv 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r3base
O=gpurun_out/r3base
timeout -k 10 400 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv1.log 2>&1 || exit 6
grep -E '^batch' $O/c4_wpv1.log
WHARF_LIB_PATH=tools/ab/lib_initstats.so timeout -k 10 400 python tools/bigscale.py --model node2vec --wpv 1 --batches 1 --mixed --no-oracle --shard 8 > $O/c4_wpv1_initstats.log 2>&1 || exit 7
grep -E 'init-stats|^batch' $O/c4_wpv1_initstats.log
timeout -k 10 600 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 > $O/c4_wpv10.log 2>&1 || exit 8
grep -E '^batch|^generate|device bytes' $O/c4_wpv10.log
