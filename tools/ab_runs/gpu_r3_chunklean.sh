#!/bin/bash
# chunk_issue in the lean form (default build) vs the round-2 form (tools/ab/lib_lean0.so): the deterministic
# suffix copy (configs[2] det probe, fused), and the node2vec plan + re-walk (configs[2] node2vec probe), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3chunklean; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paths or batch_walk_update or edge_cases or extreme or det" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
for v in lean old lean old; do
  if [ $v = old ]; then export WHARF_LIB_PATH=$PWD/tools/ab/lib_lean0.so; else unset WHARF_LIB_PATH; fi
  timeout -k 10 300 python tools/rewalk_probe.py --det --batches 4 > $O/probedet_$v.log 2>&1 || exit 6
  echo "det $v: $(tail -1 $O/probedet_$v.log)"
  timeout -k 10 300 python tools/rewalk_probe.py --model node2vec --batches 4 > $O/proben2v_$v.log 2>&1 || exit 7
  echo "n2v $v: $(tail -1 $O/proben2v_$v.log)"
done
