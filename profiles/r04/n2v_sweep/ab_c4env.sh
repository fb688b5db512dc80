set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for e in BASE=1 WHARF_N2V_LANE_SORT=0 WHARF_RET_FIRST=1 WHARF_NT_ROWS=1; do
    ( export $e; timeout -k 10 300 python -u tools/shard_balance.py --scale 26 --samples 1800000000 --model node2vec --mixed --shards 0 --blocks 16 --batches 2 ) > gpurun_out/ce_${e}_$rep.log 2>&1
    echo "c4 $e rep $rep: $(grep '^{"shard"' gpurun_out/ce_${e}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['batch_median_ms'], d['walk_update_median_ms'], d['anchor_inits_mean'])")"
  done
done
