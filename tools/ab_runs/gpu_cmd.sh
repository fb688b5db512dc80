mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -q -x -p no:cacheprovider -k "node2vec or mh or paths or shapes or shard" > gpurun_out/pt_n2v.log 2>&1; echo pytest rc=$?; tail -3 gpurun_out/pt_n2v.log
for v in base cur w4 flat; do
  lib=""; env=""
  case $v in base|w4) lib=tools/ab/lib_$v.so ;; flat) env="WHARF_N2V_REWALK=flat" ;; esac
  env $env WHARF_LIB_PATH=$lib timeout -k 10 200 python tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/ab_srt_c2_$v.log 2>&1 || exit 3
  echo c2 $v; tail -1 gpurun_out/ab_srt_c2_$v.log
  env $env WHARF_LIB_PATH=$lib timeout -k 10 400 python tools/bigscale.py --scale 24 --samples 450000000 --model node2vec --wpv 1 --batches 2 --mixed --no-oracle > gpurun_out/ab_srt_c4_$v.log 2>&1 || exit 3
  echo c4 $v; grep "^batch" gpurun_out/ab_srt_c4_$v.log
done
