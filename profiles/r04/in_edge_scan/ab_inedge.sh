set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base ie8 iep ie8p; do
    if [ $v = base ]; then unset WHARF_LIB_PATH; else export WHARF_LIB_PATH=tools/ab/lib_$v.so; fi
    timeout -k 10 300 python -u tools/shard_balance.py --shards 0 --blocks 16 --batches 3 > gpurun_out/ie_${v}_$rep.log 2>&1
    echo "c3 $v rep $rep: $(grep '^{"shard"' gpurun_out/ie_${v}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['graph_update_median_ms'], d['in_edge_scan_median_ms'], d['batch_median_ms'])")"
  done
done
unset WHARF_LIB_PATH
