#!/bin/bash
# Round-2 GPU session: parity tests, smoke, the default bench line, and a
# 2-rank gloo rehearsal of the N>1 bench path (both ranks on the one GPU).
# Every GPU step has its own time limit; a crash/abort/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py ;;
    dist2)  step bench_dist2 900 env WHARF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --rewalk-batches 5 --det-rewalk-batches 3 ;;
    c3shard8) step c3_shard8 900 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 5 --shard 8 ;;
    c4shard8) step c4_n2v_shard8 900 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 ;;
    c3det8) step c3_det_shard8 900 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 5 --det --shard 8 ;;
    abscan) for v in cur ${AB:-}; do
              lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
              step abscan_$v 600 env WHARF_LIB_PATH=$lib python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 1 --det --batches 4 --no-oracle
            done ;;
    probedet) for v in cur ${AB:-}; do
              lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
              step probedet_$v 300 env WHARF_LIB_PATH=$lib python tools/rewalk_probe.py --det --batches 3
            done ;;
    pmcdet) DET="python3 tools/rewalk_probe.py --det --batches 2"
            step pmcdet_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_rewalk_chunked" --output-format csv -d gpurun_out/pmcdet_fetch -o run -- $DET
            step pmcdet_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rewalk_chunked" --output-format csv -d gpurun_out/pmcdet_write -o run -- $DET
            step pmcdet_sq 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_rewalk_chunked" --output-format csv -d gpurun_out/pmcdet_sq -o run -- $DET
            step pmcdet_sq2 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY --kernel-include-regex "k_rewalk_chunked" --output-format csv -d gpurun_out/pmcdet_sq2 -o run -- $DET ;;
    prof)   step prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --cpu-baseline off ;;
    pmc)    GEN="python3 bench.py --steps 2 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 0 --n2v-steps 2 --n2v-rewalk-batches 0 --cpu-baseline off"
            STR="python3 bench.py --steps 1 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 3 --n2v-steps 0 --n2v-rewalk-batches 0 --cpu-baseline off"
            step pmc_gen_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_walk" --output-format csv -d gpurun_out/pmc_gen_fetch -o run -- $GEN
            step pmc_gen_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_walk" --output-format csv -d gpurun_out/pmc_gen_write -o run -- $GEN
            step pmc_str_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_rewalk_chunked|k_patch_in_edges" --output-format csv -d gpurun_out/pmc_str_fetch -o run -- $STR
            step pmc_str_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rewalk_chunked|k_patch_in_edges" --output-format csv -d gpurun_out/pmc_str_write -o run -- $STR ;;
    proben2v) for v in cur ${AB:-}; do
              lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
              step proben2v_$v 300 env WHARF_LIB_PATH=$lib python tools/rewalk_probe.py --model node2vec --batches 3
            done ;;
    pmcn2v) N2V="python3 tools/rewalk_probe.py --model node2vec --batches 2"
            step pmcn2v_tcc 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_rewalk_sorted|k_rewalk_plan|k_walk" --output-format csv -d gpurun_out/pmcn2v_tcc -o run -- $N2V
            step pmcn2v_wr 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex "k_rewalk_sorted|k_rewalk_sweep|k_walk" --output-format csv -d gpurun_out/pmcn2v_wr -o run -- $N2V
            step pmcn2v_wsize 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rewalk_sorted|k_rewalk_sweep|k_walk" --output-format csv -d gpurun_out/pmcn2v_wsize -o run -- $N2V
            step pmcdw_wr 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex "k_rewalk_sorted|k_rewalk_sweep|k_walk" --output-format csv -d gpurun_out/pmcdw_wr -o run -- python3 tools/rewalk_probe.py --batches 2
            step pmcn2v_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcn2v_trace -o run -- $N2V ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
