#!/bin/bash
# One parameterised launcher for the GPU box (replaces round 1-3's one-off
# tools/ab_runs/*.sh, kept in git history).  Run from anywhere on the box:
#   gpurun -- 'bash tools/gpu_run.sh <step> [<step> ...]'
# Steps (each under its own time limit; the script stops at the first failure):
#   tests[:<pytest -k expr>]  pytest -m gpu (optionally a subset)
#   smoke                     __graft_entry__.smoke()
#   bench[:<extra args>]      python bench.py (default line), args after ':' (use ',' for spaces)
#   rehearse                  2 gloo ranks on the one GPU: bench.py --gpus 2 at reduced scale with
#                             BASELINE's 8-GPU jobs (configs[3], configs[4]) at scale - 4
#   bigscale:<args>           tools/bigscale.py with args (',' for spaces)
#   probe:<args>              tools/rewalk_probe.py with args (',' for spaces)
#   py:<script args>          python -u <script args> (',' for spaces)
#   exe:<cmd>                 a built probe, e.g. exe:tools/sort_probe (',' for spaces)
#   rocprof:<script args>     rocprofv3 --kernel-trace --stats of python3 <script args> (',' for spaces)
#   ab:<names>                ${AB_SCRIPT:-tools/rewalk_probe.py} $PROBE_ARGS with tools/ab/lib_<name>.so per
#                             name ('base' = the tree's library), alternated twice
#   prof                      rocprofv3 kernel trace + stats of a short default bench
# Logs go to gpurun_out/<tag>_<step>.log; set TAG=... to name them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
export TMPDIR=/tmp
for step in "$@"; do
    name=${step%%:*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*:}
    args=${arg//,/ }
    log=gpurun_out/${TAG}_${name}.log
    echo "== $step -> $log"
    case $name in
    tests)
        if [ -n "$arg" ]; then
            timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
                -p no:cacheprovider -k "$arg" > "$log" 2>&1
        else
            timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
                -p no:cacheprovider > "$log" 2>&1
        fi
        rc=$?; tail -3 "$log" ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
        rc=$?; tail -1 "$log" ;;
    bench)
        timeout -k 10 900 python -u bench.py $args > "$log" 2>&1
        rc=$?
        grep '^{' "$log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'frac', d['roofline']['frac'], 'ms', d['ms_per_step'])" ;;
    rehearse)
        WHARF_DIST_BACKEND=gloo OMP_NUM_THREADS=4 timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
            --scale 20 --samples 29000000 --stream-samples 11000000 --rewalk-batches 5 --det-rewalk-batches 0 \
            --gather-probes 0 --job-scale-delta -4 --job-batches 3 $args > "$log" 2>&1
        rc=$? ;;
    bigscale)
        timeout -k 10 900 python -u tools/bigscale.py $args > "$log" 2>&1
        rc=$?; tail -2 "$log" ;;
    probe)
        timeout -k 10 900 python -u tools/rewalk_probe.py $args > "$log" 2>&1
        rc=$?; tail -4 "$log" ;;
    py)   # py:<script and args>: any python tool of the tree, output streamed to its log
        timeout -k 10 900 python -u $args > "$log" 2>&1
        rc=$?; tail -3 "$log" ;;
    exe)
        timeout -k 10 300 $args > "$log" 2>&1
        rc=$?; tail -3 "$log" ;;
    rocprof)   # rocprof:<python script and args>: kernel trace + stats of that run
        timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- python3 $args > "$log" 2>&1
        rc=$?; tail -2 "$log" ;;
    ab)   # ab:<lib1>,<lib2>,...: tools/rewalk_probe.py with each tools/ab/lib_<name>.so (base = the tree's), twice
        for rep in 1 2; do
            for item in $args; do   # <lib>[@VAR=value]: the variant's library and one environment setting
                lib=${item%%@*}; envset=""; [ "$lib" != "$item" ] && envset=${item#*@}
                if [ "$lib" = base ]; then unset WHARF_LIB_PATH; else export WHARF_LIB_PATH=tools/ab/lib_$lib.so; fi
                tag=${item//[@=]/_}
                ( [ -n "$envset" ] && export "$envset"; timeout -k 10 600 python -u ${AB_SCRIPT:-tools/rewalk_probe.py} $PROBE_ARGS ) \
                    > gpurun_out/${TAG}_ab_${tag}_$rep.log 2>&1
                rc=$?; echo "$item rep $rep: $(tail -1 gpurun_out/${TAG}_ab_${tag}_$rep.log)"
                [ $rc -eq 0 ] || exit $rc
            done
        done
        unset WHARF_LIB_PATH ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- \
            python3 bench.py --steps 5 --warmup 2 --rewalk-batches 10 --det-rewalk-batches 10 --n2v-steps 0 \
            --per-gpu-of-8 0 --cpu-baseline off --gather-probes 0 > "$log" 2>&1
        rc=$? ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
    echo "== $step rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
