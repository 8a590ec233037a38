#!/bin/bash
# Sort change check in one GPU call: the GPU suite, the sort micro-benchmark and phase trace at the
# headline and config-5 sizes, then a 1-stream A/B against LIB_BASE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SORT_LARGE=1 timeout -k 10 200 python scripts/sort_bench.py > $OUT/sort_bench.log 2>&1; rc=$?; cat $OUT/sort_bench.log | grep ms; [ $rc -eq 0 ] || exit $rc
SORT_LARGE=1 GSR_LIB_PATH=$PWD/sdp-gs_amd/gsr_amd/libgsr_trace.so timeout -k 10 200 python scripts/sort_trace.py > $OUT/sort_trace.json 2> $OUT/sort_trace.err; rc=$?
python3 -c "
import json;d=json.load(open('$OUT/sort_trace.json'))
for k,v in d.items(): print(k, v['parts'], 'end', v['end_us_q'], 'lookback', v['lookback_us_q'], 'rank', v['rank_us_q'])
"; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 LIBS="${LIB_BASE:-libgsr_base.so} libgsr.so" BENCH_ARGS="--streams 1" bash scripts/ab_parity.sh
