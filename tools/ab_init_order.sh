#!/bin/bash
# Same-box A/B of the configs[4] shard's first generation (node2vec MH WEIGHT, every anchor computed
# up front) across init-order variants, alternated REPS times:
#   hybrid  the tree's library (two orders by the line model)
#   prev    the tree's library, WHARF_INIT_ORDER=0 (prev order only)
#   lib:<n> tools/ab/lib_<n>.so (e.g. an older build)
#   bias:<x> the tree's library, WHARF_INIT_CUR_BIAS=x (lines added to the cur-order side)
#   env:<VAR=v> the tree's library with one environment setting
# Logs: gpurun_out/${TAG:-initord}_<variant>_<rep>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-initord}
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
    for v in "$@"; do
        log=gpurun_out/${TAG}_$(echo "$v" | tr ":=/" "___")_${rep}.log
        (
            case $v in
                prev) export WHARF_INIT_ORDER=0 ;;
                lib:*) export WHARF_LIB_PATH=tools/ab/lib_${v#lib:}.so ;;
                bias:*) export WHARF_INIT_CUR_BIAS=${v#bias:} ;;
                env:*) export "${v#env:}" ;;
            esac
            timeout -k 10 300 python -u tools/bigscale.py --model node2vec --wpv 10 --batches ${BATCHES:-2} --mixed \
                --no-oracle --shard 8
        ) > "$log" 2>&1
        rc=$?
        echo "== $v rep $rep rc=$rc: $(grep -o '"first_gen_ms": [0-9.]*\|"gen_ms": [0-9.]*\|"batch_median_ms": [0-9.]*\|"first_gen_anchor_inits": [0-9]*' "$log" | tr '\n' ' ')"
        [ $rc -eq 0 ] || exit $rc
    done
done
