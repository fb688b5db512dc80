#!/bin/bash
# Per-lane WEIGHT init in k_anchor_init_all: node2vec parity, then first generation A/B (tools/ab variants) + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -m gpu -q -x \
  -k "node2vec or mh" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_initall.log 2>&1
rc=$?; tail -2 gpurun_out/pt_initall.log; [ $rc -eq 0 ] || exit $rc
AB="${AB:-}" bash tools/ab_runs/gpu_genpre_ab.sh
