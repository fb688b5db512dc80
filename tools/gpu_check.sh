#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench.  Every GPU step has
# its own time limit; a crash/abort/timeout ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench18) step bench_s18 600 python bench.py --scale 18 --samples 7324270 --steps 3 --warmup 1 --cpu-baseline off ;;
    bench)  step bench 900 python bench.py ;;
    benchq) step benchq 600 python bench.py --cpu-baseline off ;;
    rwsweep) for b in 0 8 16 32 64; do
               step rw_bpc$b 600 env WHARF_WALK_BLOCKS_PER_CU=$b python bench.py --steps 2 --warmup 1 --rewalk-batches 10 --cpu-baseline off
             done ;;
    lssweep) for t in 0 8 16 24 40 65; do
               step ls_c3_dw_$t 300 env WHARF_LOCKSTEP_MIN=$t python tools/rewalk_probe.py --batches 3
               step ls_c3_n2v_$t 300 env WHARF_LOCKSTEP_MIN=$t python tools/rewalk_probe.py --batches 3 --model node2vec
             done
             for t in 0 16 40 65; do
               step ls_c4_$t 600 env WHARF_LOCKSTEP_MIN=$t python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 2 --no-oracle
               step ls_c5_$t 600 env WHARF_LOCKSTEP_MIN=$t python tools/bigscale.py --model node2vec --wpv 1 --batches 2 --mixed
             done ;;
    roof)   step gather_roof 300 tools/gather_roof 3.48 ;;
    roofcal) for m in dep dep_64B_block dep_128B_block; do
              step roofcal_$m 120 tools/gather_roof 3.48 coarse $m
              step roofcal_fetch_$m 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/roofcal_fetch_$m -o run -- tools/gather_roof 3.48 coarse $m
              step roofcal_req_$m 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/roofcal_req_$m -o run -- tools/gather_roof 3.48 coarse $m
            done ;;
    big)    step bigscale 900 python tools/bigscale.py ;;
    index)  step index_probe 800 python tools/index_probe.py ;;
    c4)     step c4_stream 1100 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 50 ;;
    c4det)  step c4_det 1100 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 10 --det ;;
    c5n2v)  step c5_node2vec 1100 python tools/bigscale.py --model node2vec --wpv 1 --batches 10 --mixed ;;
    detnm)  step bench_det_nomemo 900 env WHARF_NO_MEMO=1 python bench.py --det --steps 3 --warmup 1 --rewalk-batches 5 --cpu-baseline off ;;
    chunk)  step probe_det 300 python tools/rewalk_probe.py --det --batches 3
            step probe_det_nochunk 300 env WHARF_NO_CHUNKED_SCAN=1 python tools/rewalk_probe.py --det --batches 3
            step probe_mh 300 python tools/rewalk_probe.py --batches 3
            step probe_mh_nochunk 300 env WHARF_NO_CHUNKED_SCAN=1 python tools/rewalk_probe.py --batches 3 ;;
    ab)     for v in cur ${AB:-$(ls tools/ab 2>/dev/null | sed -n 's/^lib_\(.*\)\.so$/\1/p')}; do
              lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
              step ab_${ABTAG:-det}_$v 300 env WHARF_LIB_PATH=$lib python tools/rewalk_probe.py ${PROBE:---det --batches 3}
            done ;;
    n2vinit) for i in random burnin weight; do
              step n2v_init_$i 300 python tools/rewalk_probe.py --model node2vec --batches 3 --init $i
            done
            step n2v_q1 300 python tools/rewalk_probe.py --model node2vec --batches 3 --p 4 --q 1 ;;
    abn2v)  for v in cur ${AB:-}; do
              lib=""; [ $v = cur ] || lib=tools/ab/lib_$v.so
              step abn2v_$v 600 env WHARF_LIB_PATH=$lib python bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 3 --det-rewalk-batches 0 --cpu-baseline off
            done ;;
    det)    step bench_det 900 python bench.py --det --steps 3 --warmup 1 --rewalk-batches 5 --cpu-baseline off ;;
    n2vnf)  step bench_n2v_nofilter 900 env WHARF_NO_NEIGHBOUR_FILTER=1 python bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 5 --cpu-baseline off ;;
    c5n2vnf) step c5_node2vec_nofilter 1100 env WHARF_NO_NEIGHBOUR_FILTER=1 python tools/bigscale.py --model node2vec --wpv 1 --batches 4 --mixed --no-oracle ;;
    c5n2vq) step c5_node2vec_q 1100 python tools/bigscale.py --model node2vec --wpv 1 --batches 4 --mixed --no-oracle ;;
    n2v)    step bench_n2v 900 python bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 5 --cpu-baseline off ;;
    dist2)  step bench_dist2 900 env WHARF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scale 20 --samples 29296270 --stream-samples 10000000 --steps 3 --warmup 1 --rewalk-batches 5 ;;
    dist4)  step bench_dist4 900 env WHARF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --scale 20 --samples 29296270 --stream-samples 10000000 --steps 3 --warmup 1 --rewalk-batches 5 --det-rewalk-batches 3 ;;
    dist2full) step bench_dist2_full 900 env WHARF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --rewalk-batches 5 ;;
    prof)   step prof_gen 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off ;;
    pmc)    step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --rewalk-batches 0 --cpu-baseline off
            step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 0 --rewalk-batches 0 --cpu-baseline off
            step pmc_req 900 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_req -o run -- python3 bench.py --steps 2 --warmup 0 --rewalk-batches 0 --cpu-baseline off ;;
    profdet) DET="python3 tools/rewalk_probe.py --det --batches 3"
            step det_probe 300 $DET
            step det_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/det_trace -o run -- $DET
            step det_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/det_fetch -o run -- $DET
            step det_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/det_write -o run -- $DET
            step det_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/det_tcc -o run -- $DET ;;
    pmcn2v) N2V="python3 bench.py --model node2vec --steps 2 --warmup 1 --rewalk-batches 0 --cpu-baseline off"
            step n2v_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/n2v_trace -o run -- $N2V
            step n2v_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/n2v_fetch -o run -- $N2V
            step n2v_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/n2v_write -o run -- $N2V ;;
  esac
done
