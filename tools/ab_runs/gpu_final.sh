#!/bin/bash
# Parity subset for the re-walk kernels, the deterministic probe, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "paths or det" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_final.log 2>&1
rc=$?; tail -2 gpurun_out/pt_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/rewalk_probe.py --det --batches 3 > gpurun_out/probedet_final.log 2>&1 || exit 6
grep -E "^batch" gpurun_out/probedet_final.log
timeout -k 10 900 python bench.py > gpurun_out/bench_final.log 2>&1 || exit 7
python - gpurun_out/bench_final.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
n = d["mh_node2vec"]; r = d["rewalk_latency_10k_batch"]; t = d["rewalk_latency_10k_batch_deterministic"]
print("value", d["value"], "frac", d["roofline"]["frac"], "ceiling", d["roofline"]["gather_ceiling"])
print("n2v warm", n["warm_generation_kernel_ms"], "first", n["first_generation_kernel_ms"], "batch", n["rewalk_latency_10k_batch"]["median_ms"])
print("mh batch", r["median_ms"], "det batch", t["median_ms"], t["median_rewalk_kernel_ms"], "scan", t["scan_only_median_ms"])
PY
