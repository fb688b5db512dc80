#!/bin/bash
# DeepWalk MH generation: 16-B edge records (default) vs the 4-B target + the target's vertex row
# (WHARF_GEN_ADJ=1, an A/B switch since removed: 118 vs 80 ms): parity, then configs[1] generation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3genadj; mkdir -p $O
WHARF_GEN_ADJ=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "rmat10 or wiki or deepwalk or stream" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pt.log 2>&1
rc=$?; grep -E "passed|failed" $O/pt.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pt.log | head; exit $rc; }
Q="--steps 10 --warmup 2 --rewalk-batches 0 --det-rewalk-batches 0 --cpu-baseline off --n2v-steps 0 --n2v-rewalk-batches 0 --per-gpu-of-8 0 --gather-probes 1"
for v in 1 0 1 0 1 0; do
  WHARF_GEN_ADJ=$v timeout -k 10 300 python bench.py $Q > $O/b_$v.log 2>&1 || exit 6
  echo "gen_adj=$v: $(tail -1 $O/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
