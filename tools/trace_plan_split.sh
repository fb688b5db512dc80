#!/bin/bash
# Kernel traces of the node2vec plan split (default) vs fused (WHARF_PLAN_SPLIT=0) on the configs[4]
# shard and the configs[2] graph, alternated twice: gpurun_out/plansplit/<case>_<variant>_<rep>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/plansplit
mkdir -p $O
C4="python3 tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8"
C2="python3 tools/bigscale.py --scale 22 --samples 43000000 --model node2vec --wpv 10 --batches 4 --no-oracle"
for rep in 1 2; do
    for v in split fused; do
        for c in c4 c2; do
            cmd=$C4; [ $c = c2 ] && cmd=$C2
            sp=1; [ $v = fused ] && sp=0
            WHARF_PLAN_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${c}_${v}_$rep -o run -- $cmd \
                > $O/${c}_${v}_$rep.log 2>&1 || exit $?
            echo "done $c $v $rep"
        done
    done
done
