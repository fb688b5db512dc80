#!/bin/bash
# Pre-init proposal rounds A/B (first node2vec generation, configs[2] batches) + kernel trace of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 3 --det-rewalk-batches 0 --cpu-baseline off"
for v in cur ${AB:-}; do
  lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
  WHARF_LIB_PATH=$lib timeout -k 10 400 $B > gpurun_out/genpre_ab_$v.log 2>&1 || exit 6
  echo $v; python - gpurun_out/genpre_ab_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]; w = d["rewalk_latency_10k_batch"]
print("first", r["first_generation_kernel_ms"], "warm", r["avg_kernel_ms"], "batch", w["median_ms"], w["median_rewalk_kernel_ms"])
PY
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_genpre -o run -- $B > gpurun_out/prof_genpre.log 2>&1 || exit 7
find gpurun_out/prof_genpre -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-160
