#!/bin/bash
# Load balance of the 8-GPU jobs: the per-GPU work of ranks 0, 3 and 7 (start-vertex shards of
# balanced_shards) for configs[3] DeepWalk MH and configs[4] node2vec (wpv 10); the job's batch time is the
# max over ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3shards; mkdir -p $O
for i in 0 3 7; do
  timeout -k 10 400 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --shard 8 --shard-index $i --batches 5 --no-oracle > $O/c3_mh_shard${i}.log 2>&1 || exit 6
  echo "c3 mh shard $i: $(grep -E '^shard|^generate' $O/c3_mh_shard${i}.log | cut -c1-110 | tr '\n' ' ') | $(grep '^{' $O/c3_mh_shard${i}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["batch_median_ms"], d["graph_update_median_ms"], d["walk_update_median_ms"], d["mean_affected"], d["mean_rewalk_steps"], d["rewalk_Gsteps_per_s"])')"
done
for i in 0 7; do
  timeout -k 10 400 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 --shard-index $i > $O/c4_n2v_shard${i}.log 2>&1 || exit 7
  echo "c4 n2v shard $i: $(grep '^{' $O/c4_n2v_shard${i}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gen_ms"], d["first_gen_ms"], d["batch_median_ms"], d["graph_update_median_ms"], d["walk_update_median_ms"], d["mean_affected"], d["mean_rewalk_steps"], d["rewalk_Gsteps_per_s"], d["mean_anchor_inits"])')"
done
