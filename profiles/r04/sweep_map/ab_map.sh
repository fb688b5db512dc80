set -e
mkdir -p gpurun_out
for rep in 1 2; do
  (cd tools/ab/r03 && timeout -k 10 300 python -u tools/rewalk_probe.py --batches 6) > gpurun_out/rm_r03_$rep.log 2>&1
  echo "r03 rep $rep: $(tail -1 gpurun_out/rm_r03_$rep.log | cut -c1-100)"
  timeout -k 10 300 python -u tools/rewalk_probe.py --batches 6 > gpurun_out/rm_head_$rep.log 2>&1
  echo "head rep $rep: $(tail -1 gpurun_out/rm_head_$rep.log | cut -c1-100)"
  WHARF_LIB_PATH=tools/ab/lib_oldmap.so timeout -k 10 300 python -u tools/rewalk_probe.py --batches 6 > gpurun_out/rm_oldmap_$rep.log 2>&1
  echo "oldmap rep $rep: $(tail -1 gpurun_out/rm_oldmap_$rep.log | cut -c1-100)"
done
for k in ranges blocks; do
  if [ $k = blocks ]; then B="--blocks 16"; else B=""; fi
  timeout -k 10 300 python -u tools/shard_balance.py --shards 0 3 0 3 $B > gpurun_out/rm_c3_$k.log 2>&1
  echo "c3 $k: $(grep '^{"shard"' gpurun_out/rm_c3_$k.log | python -c "import sys,json; print([json.loads(l)['walk_update_median_ms'] for l in sys.stdin])")"
done
