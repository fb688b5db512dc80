#!/bin/bash
# Cold-cache anchor init for node2vec generation: parity, then first/warm generation with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_fullsize.py -m gpu -q -x \
  -k "node2vec or paths or mh or shard" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_genpre.log 2>&1
rc=$?; tail -3 gpurun_out/pt_genpre.log; [ $rc -eq 0 ] || exit $rc
for v in pre lazy; do
  np=0; [ $v = lazy ] && np=1
  WHARF_NO_PREINIT=$np timeout -k 10 400 python bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 3 --det-rewalk-batches 0 --cpu-baseline off > gpurun_out/genpre_$v.log 2>&1 || exit 6
  echo $v; python - gpurun_out/genpre_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]; w = d["rewalk_latency_10k_batch"]
print("first", r["first_generation_kernel_ms"], "warm", r["avg_kernel_ms"], "value", d["value"], "batch", w["median_ms"], w["median_rewalk_kernel_ms"])
PY
done
