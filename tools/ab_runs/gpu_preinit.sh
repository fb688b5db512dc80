#!/bin/bash
# Anchor pre-init: node2vec parity tests, then the configs[2] node2vec re-walk with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -m gpu -q -x \
  -k "node2vec or paths or mh or shard" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_preinit.log 2>&1
rc=$?; tail -3 gpurun_out/pt_preinit.log; [ $rc -eq 0 ] || exit $rc
for v in pre lazy pre2; do
  np=0; [ $v = lazy ] && np=1
  WHARF_NO_PREINIT=$np timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/preinit_c2_$v.log 2>&1 || exit 6
  echo $v; grep -E "^batch|^\{" gpurun_out/preinit_c2_$v.log
done
