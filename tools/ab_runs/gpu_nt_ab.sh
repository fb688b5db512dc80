#!/bin/bash
# Non-temporal walk-matrix loads/stores in the chunked scans: configs[2] det + node2vec probes and configs[3] 1/8-shard det, alternating variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
i=0
for v in cur nt0 nt2 cur nt0 nt2; do
  i=$((i+1)); lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
  WHARF_LIB_PATH=$lib timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > gpurun_out/nt_c2det_${v}_$i.log 2>&1 || exit 6
  echo "c2det $v: $(tail -1 gpurun_out/nt_c2det_${v}_$i.log)"
  WHARF_LIB_PATH=$lib timeout -k 10 300 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 4 --det --shard 8 --no-oracle > gpurun_out/nt_c3det_${v}_$i.log 2>&1 || exit 6
  echo "c3det $v: $(grep -E '^batch' gpurun_out/nt_c3det_${v}_$i.log | sed 's/, affected.*//;s/batch [0-9]: //' | tr '\n' ' ')"
done
for v in cur nt0 cur nt0; do
  i=$((i+1)); lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
  WHARF_LIB_PATH=$lib timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 3 > gpurun_out/nt_c2n2v_${v}_$i.log 2>&1 || exit 6
  echo "c2n2v $v: $(tail -1 gpurun_out/nt_c2n2v_${v}_$i.log)"
done
