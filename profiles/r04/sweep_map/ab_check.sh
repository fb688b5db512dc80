set -e
mkdir -p gpurun_out
TAG=h1 bash tools/gpu_run.sh tests:shards\ or\ distributed\ or\ paths\ or\ golden\ or\ walk_rows\ or\ fullsize
timeout -k 10 300 python -u tools/rewalk_probe.py --batches 6 > gpurun_out/hc_head.log 2>&1
echo "head: $(tail -1 gpurun_out/hc_head.log | cut -c1-100)"
for k in ranges blocks; do
  if [ $k = blocks ]; then B="--blocks 16"; else B=""; fi
  timeout -k 10 300 python -u tools/shard_balance.py --shards 0 3 0 3 $B > gpurun_out/hc_c3_$k.log 2>&1
  echo "c3 $k: $(grep '^{"shard"' gpurun_out/hc_c3_$k.log | python -c "import sys,json; print([json.loads(l)['walk_update_median_ms'] for l in sys.stdin])")"
done
timeout -k 10 300 python -u tools/shard_balance.py --scale 26 --samples 1800000000 --model node2vec --mixed --shards 0 --blocks 16 --batches 3 > gpurun_out/hc_c4.log 2>&1
echo "c4: $(grep '^{"shard"' gpurun_out/hc_c4.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['batch_median_ms'], d['walk_update_median_ms'], d['first_generation_ms'])")"
