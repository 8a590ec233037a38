#!/bin/bash
# One GPU-box session: GPU tests -> bench -> rocprofv3 kernel-trace stats.
# Stops at the first step that ends abnormally (fault / abort / segfault / timeout); an ordinary
# test failure (exit 1) still lets the bench run so one call yields both pieces of evidence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
abnormal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  if abnormal $rc; then echo "stopping after abnormal pytest exit"; exit $rc; fi
fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stage-timing ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
  find $OUT/prof -name "*stats*" | head
fi
