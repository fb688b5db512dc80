set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/pt_dist.log 2>&1 || exit 5
tail -2 gpurun_out/pt_dist.log
for i in random weight; do
  timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 --init $i > gpurun_out/n2v_init_$i.log 2>&1 || exit 6
  tail -2 gpurun_out/n2v_init_$i.log
done
WHARF_LIB_PATH=tools/ab/lib_initstats.so timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/n2v_initstats.log 2>&1 || exit 7
grep init-stats gpurun_out/n2v_initstats.log | tail -4
