#!/bin/bash
# SQ counters of the deterministic suffix copy (k_rewalk_chunked<true>) and the lean scan on configs[2] (det probe).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r3copypmc; mkdir -p $O
export TMPDIR=/tmp
P="python3 tools/rewalk_probe.py --det --batches 2"
R="k_rewalk_chunked|k_rewalk_scan"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR --kernel-include-regex "$R" --output-format csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 || { echo "pmc1 failed"; exit 6; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$R" --output-format csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 || { echo "pmc2 failed"; exit 7; }
echo done
