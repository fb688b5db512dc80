#!/bin/bash
# Pre-init only when the walks are dense in the states: node2vec parity, then configs[4] 1/8 shard (rule: lazy) vs forced pre-init, configs[2] node2vec probe (rule: pre-init).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x -k "node2vec or paths" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_prerule.log 2>&1
rc=$?; tail -2 gpurun_out/pt_prerule.log; [ $rc -eq 0 ] || exit $rc
for v in rule forced rule forced; do
  np=""; [ $v = forced ] && np=0
  WHARF_NO_PREINIT=$np timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > gpurun_out/prerule_c4_$v.log 2>&1 || exit 6
  echo "c4n2v $v: $(grep -E '^batch' gpurun_out/prerule_c4_$v.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
done
timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/prerule_c2n2v.log 2>&1 || exit 6
echo "c2n2v rule: $(tail -1 gpurun_out/prerule_c2n2v.log)"
