#!/bin/bash
# GPU session steps (OUTDIR=gpurun_out/r4 for round 4; default gpurun_out/r3) (each with its own time limit; a crash/abort/timeout ends the session):
#   pytest smoke bench prof pmc c4w10 c4w1 c3shard8 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUTDIR=${OUTDIR:-gpurun_out/r3}
mkdir -p ${OUTDIR}
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "${OUTDIR}/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "${OUTDIR}/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py ;;
    prof)   step prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUTDIR}/prof_bench -o run -- python3 bench.py --cpu-baseline off ;;
    pmc)    GEN="python3 bench.py --steps 2 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 0 --n2v-steps 2 --n2v-rewalk-batches 0 --cpu-baseline off --per-gpu-of-8 0 --gather-probes 0"
            STR="python3 bench.py --steps 1 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 3 --n2v-steps 0 --n2v-rewalk-batches 0 --cpu-baseline off --per-gpu-of-8 0 --gather-probes 0"
            step pmc_gen_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_walk" --output-format csv -d ${OUTDIR}/pmc_gen_fetch -o run -- $GEN
            step pmc_gen_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_walk" --output-format csv -d ${OUTDIR}/pmc_gen_write -o run -- $GEN
            step pmc_str_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_rewalk_chunked|k_rewalk_scan|k_patch_in_edges|k_patch_rev" --output-format csv -d ${OUTDIR}/pmc_str_fetch -o run -- $STR
            step pmc_str_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rewalk_chunked|k_rewalk_scan|k_patch_in_edges|k_patch_rev" --output-format csv -d ${OUTDIR}/pmc_str_write -o run -- $STR
            # durations of exactly the launches the streaming PMC passes count
            step prof_str 600 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUTDIR}/prof_str -o run -- $STR ;;
    pmcstr) STR="python3 bench.py --steps 1 --warmup 0 --rewalk-batches 0 --det-rewalk-batches 3 --n2v-steps 0 --n2v-rewalk-batches 0 --cpu-baseline off --per-gpu-of-8 0 --gather-probes 0"
            step pmc_str_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_rewalk_chunked|k_rewalk_scan|k_patch_in_edges|k_patch_rev" --output-format csv -d ${OUTDIR}/pmc_str_fetch -o run -- $STR
            step pmc_str_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rewalk_chunked|k_rewalk_scan|k_patch_in_edges|k_patch_rev" --output-format csv -d ${OUTDIR}/pmc_str_write -o run -- $STR
            step prof_str 600 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUTDIR}/prof_str -o run -- $STR ;;
    c4w10)  step c4_n2v_wpv10_shard8 600 python tools/bigscale.py --model node2vec --wpv 10 --batches 3 --mixed --no-oracle --shard 8 ;;
    c4w1)   step c4_n2v_wpv1_shard8 600 python tools/bigscale.py --model node2vec --wpv 1 --batches 3 --mixed --no-oracle --shard 8 ;;
    c3shard8) step c3_shard8 900 python tools/bigscale.py --scale 25 --samples 1200000000 --wpv 10 --batches 5 --shard 8 ;;
    readout) step walk_readout 400 tools/walk_readout 20000 41943040 ;;
    c4pmc)  C4="python3 tools/bigscale.py --model node2vec --wpv 10 --batches 2 --mixed --no-oracle --shard 8"
            R="k_rewalk_sorted|k_rewalk_plan|k_anchor|k_patch_in_edges|k_walk"
            step c4_trace 600 rocprofv3 --kernel-trace --stats --kernel-include-regex "$R" --output-format csv -d ${OUTDIR}/c4_trace -o run -- $C4
            step c4_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" --output-format csv -d ${OUTDIR}/c4_fetch -o run -- $C4
            step c4_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" --output-format csv -d ${OUTDIR}/c4_write -o run -- $C4 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
