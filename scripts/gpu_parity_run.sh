#!/bin/bash
# One GPU call: activation probe, the benchmarked path vs the oracle (tests/test_fused_parity.py),
# then the rest of the GPU suite and a short bench.  Each step has its own time limit; the call
# stops at the first abnormal exit (fault / abort / time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
abnormal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 300 python -u scripts/probe_activations.py > gpurun_out/probe.json 2> gpurun_out/probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/probe.json; tail -3 gpurun_out/probe.err; abnormal $rc && exit $rc
timeout -k 10 ${PARITY_TIMEOUT:-900} python -u -m pytest -v -s --timeout 900 --timeout-method thread tests/test_fused_parity.py -m gpu ${PARITY_ARGS:-} > gpurun_out/fused_parity.log 2>&1
rc=$?; echo "fused parity rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/fused_parity.log | tail -20; abnormal $rc && exit $rc
if [ "${REST:-1}" = "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu --deselect tests/test_fused_parity.py ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; abnormal $rc && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; exit $rc
