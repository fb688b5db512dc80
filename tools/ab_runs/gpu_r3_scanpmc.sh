#!/bin/bash
# Rewalk-point scan kernels on configs[2] (deterministic probe, 2 batches): kernel trace + two SQ counter
# passes per variant (first / big / pipe16), to see where each spends its cycles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3scanpmc; mkdir -p $O
P="python3 tools/rewalk_probe.py --det --batches 2"
R="k_rewalk_scan|k_rewalk_chunked"
for v in first big pipe16; do
  unset WHARF_SCAN_SMALL_BLOOM
  export WHARF_SCAN_KERNEL=$v
  [ $v = pipe16 ] && { export WHARF_SCAN_KERNEL=pipe; export WHARF_SCAN_SMALL_BLOOM=1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$R" --output-format csv -d $O/tr_$v -o run -- $P > $O/tr_$v.log 2>&1 || { echo "trace $v failed"; exit 5; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$R" --output-format csv -d $O/p1_$v -o run -- $P > $O/p1_$v.log 2>&1 || { echo "pmc1 $v failed"; exit 6; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$R" --output-format csv -d $O/p2_$v -o run -- $P > $O/p2_$v.log 2>&1 || { echo "pmc2 $v failed"; exit 7; }
  echo "$v done"
done
