set -e
mkdir -p gpurun_out
WHARF_START_PREINIT=1 TAG=sp bash tools/gpu_run.sh tests:node2vec
for rep in 1 2; do
  for v in 0 1; do
    WHARF_START_PREINIT=$v timeout -k 10 300 python -u tools/shard_balance.py --scale 26 --samples 1800000000 --model node2vec --mixed --shards 0 --blocks 16 --batches 2 > gpurun_out/sp_${v}_$rep.log 2>&1
    echo "c4 start_pre=$v rep $rep: $(grep '^{"shard"' gpurun_out/sp_${v}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['batch_median_ms'], d['walk_update_median_ms'], d['anchor_inits_mean'], d['batch_ms'])")"
  done
done
