#!/bin/bash
# Quick GPU iteration: GPU tests (optionally a subset) then bench at 1 and 2 streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests} -m gpu > gpurun_out/t_quick.log 2>&1; rc=$?; tail -4 gpurun_out/t_quick.log; [ $rc -le 1 ] || exit $rc
for s in ${STREAMS:-1 2}; do timeout -k 10 300 python bench.py --streams $s --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_s$s.json 2> gpurun_out/b_s$s.err || exit $?; python -c "import json;d=json.load(open('gpurun_out/b_s$s.json'));print($s, d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
