#!/bin/bash
# Full GPU check of the tree as built: gpu tests, smoke, default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_check.log 2>&1
rc=$?; tail -3 gpurun_out/pt_check.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_check.log 2>&1 || exit 5
tail -1 gpurun_out/smoke_check.log
timeout -k 10 900 python bench.py > gpurun_out/bench_check.log 2>&1 || exit 7
grep '^{' gpurun_out/bench_check.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'frac', d['roofline']['frac'], 'ms', d['ms_per_step'])"
