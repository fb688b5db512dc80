#!/bin/bash
# Per-batch choice of non-temporal row loads in the chunked scans: parity (paths with both choices), then configs[2] det / node2vec probes and configs[3] 1/8-shard det with the host's choice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "paths or det" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_ntrows.log 2>&1
rc=$?; tail -2 gpurun_out/pt_ntrows.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > gpurun_out/ntrows_c2det_$i.log 2>&1 || exit 6
  echo "c2det: $(tail -1 gpurun_out/ntrows_c2det_$i.log)"
  timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --det --shard 8 --no-oracle > gpurun_out/ntrows_c3det_$i.log 2>&1 || exit 6
  echo "c3det: $(grep -E '^batch' gpurun_out/ntrows_c3det_$i.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
done
timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 5 --shard 8 > gpurun_out/ntrows_c3mh.log 2>&1 || exit 6
echo "c3mh: $(grep -E '^batch' gpurun_out/ntrows_c3mh.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
timeout -k 10 300 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 > gpurun_out/ntrows_c4n2v.log 2>&1 || exit 6
echo "c4n2v: $(grep -E '^batch' gpurun_out/ntrows_c4n2v.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
