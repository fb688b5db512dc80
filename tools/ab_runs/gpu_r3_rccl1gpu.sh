#!/bin/bash
# Round 3: the N>1 bench path over RCCL (backend "nccl") with 2 ranks sharing the one GPU of the box
# (a rehearsal of the driver's 8-GPU run: init_process_group(device_id), all_reduce of the counters,
# batch_isend_irecv corpus all-gatherv on device tensors).  Small graph; everything under a time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/rccl1gpu; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --scale 18 --samples 2000000 --stream-samples 1000000 --steps 3 --warmup 1 \
  --rewalk-batches 3 --det-rewalk-batches 2 --gather-probes 0 --per-gpu-of-8 0 --n2v-steps 0 --cpu-baseline off \
  > $O/bench_nccl_2ranks.log 2>&1
rc=$?; tail -5 $O/bench_nccl_2ranks.log; exit $rc
