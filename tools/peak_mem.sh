#!/bin/bash
# The 8-GPU jobs' per-rank peak on ONE GPU: bench.py --init-dist (a process group
# of one over RCCL) with BASELINE's jobs at full scale.  configs[4] runs its rank-0 share (walk shard 0
# of 8: the per-rank load of the 8-GPU job), builds the graph, every anchor, the reverse index, the
# bounded gather with RCCL buffers live and the insert/delete pairs; configs[3] at world 1 holds every
# walk.  jobs_8gpu.<job>.device_memory = the lowest hipMemGetInfo free seen.
#   gpurun -- 'bash tools/peak_mem.sh [extra bench args]'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
log=gpurun_out/${TAG:-peak}_peak_mem.log
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --init-dist --steps 1 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 0 \
    --n2v-steps 0 --per-gpu-of-8 0 --cpu-baseline off --gather-probes 0 --jobs configs3,configs4 --job-batches 2 \
    "$@" > "$log" 2>&1
rc=$?
echo "== peak_mem rc=$rc"
python - "$log" <<'PYEOF'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        for k, j in (d.get('jobs_8gpu') or {}).items():
            g = j.get('corpus_allgatherv') or {}
            print(k, 'error' if 'error' in j else 'ok', j.get('error', ''), json.dumps(j.get('device_memory')),
                  'checksum_ok', g.get('checksum_of_checksums_ok'), 'batch_median_ms', j.get('batch_median_ms'),
                  'first_gen_ms', j.get('first_generation_ms'))
PYEOF
exit $rc
