#!/bin/bash
# Same-box A/B of bench.py's per_gpu_of_8 cases (configs[3] shard 0 of 8, configs[3] all walks on one GPU,
# configs[4] node2vec shard 0 of 8), alternated REPS times over the variants named on the command line:
#   head         this tree, defaults
#   head@VAR=v   this tree with one environment setting (e.g. head@WHARF_REV=0)
#   tree:<dir>   another tree's bench.py + package (e.g. tools/ab/r04, built from an older commit)
# Logs: gpurun_out/${TAG:-per8}_<variant>_<rep>.log; a failing run ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-per8}
REPS=${REPS:-2}
ARGS="--steps 1 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 0 --n2v-steps 0 --cpu-baseline off --gather-probes 0 ${EXTRA:-}"
for rep in $(seq 1 $REPS); do
    for v in "$@"; do
        name=${v%%@*}; envset=""; [ "$name" != "$v" ] && envset=${v#*@}
        dir=.; case $name in tree:*) dir=${name#tree:};; esac
        tag=$(echo "$v" | tr '@=:/' '____')
        log=gpurun_out/${TAG}_${tag}_${rep}.log
        ( [ -n "$envset" ] && export "$envset"; cd "$dir" && timeout -k 10 420 python -u bench.py $ARGS ) > "$log" 2>&1
        rc=$?
        echo "== $v rep $rep rc=$rc"
        python - "$log" <<'PYEOF'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('per_gpu_of_8 ') and ': {' in l:
        k, j = l.split(': ', 1); d = json.loads(j)
        print(k[13:], {x: d.get(x) for x in ('first_generation_ms', 'generation_ms', 'batch_median_ms', 'graph_update_median_ms', 'walk_update_median_ms', 'rewalk_kernel_median_ms', 'mean_anchor_inits', 'in_edge_records', 'device_bytes')})
    elif l.startswith('{'):
        d = json.loads(l)
        n2v = d.get('mh_node2vec') or {}
        rw = n2v.get('rewalk_latency_10k_batch') or {}
        print('headline', d.get('value'), 'mh_node2vec first/warm gen ms', n2v.get('first_generation_kernel_ms'),
              n2v.get('warm_generation_kernel_ms'), 'n2v rewalk median ms', rw.get('median_ms'))
        c2, c2d = d.get('rewalk_latency_10k_batch') or {}, d.get('rewalk_latency_10k_batch_deterministic') or {}
        probes = ((d.get('roofline') or {}).get('gather_ceiling') or {}).get('probes')
        print('configs2 MH / det median ms', c2.get('median_ms'), c2d.get('median_ms'), 'rewalk kernel',
              c2.get('median_rewalk_kernel_ms'), c2d.get('median_rewalk_kernel_ms'), 'gen same graph',
              (c2.get('generation_same_graph') or {}).get('ms'), 'probes', probes)
PYEOF
        [ $rc -eq 0 ] || exit $rc
    done
done
