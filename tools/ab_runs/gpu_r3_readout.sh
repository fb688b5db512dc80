#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3readout; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "snapshot or golden or shards" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pt.log | head; exit $rc; }
timeout -k 10 400 tools/walk_readout 20000 41943040 > $O/walk_readout.log 2>&1 || exit 6
cat $O/walk_readout.log
