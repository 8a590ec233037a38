#!/bin/bash
# GPU suite on the default build (stops on any failure), then alternating bench runs of
# library / env variants at 1 and 3 streams.
# usage: VARIANTS="NONE=1 GSR_LIB_PATH=sdp-gs_amd/gsr_amd/libgsr_x.so" [STREAMS="1 3"] bash scripts/r03_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > $OUT/t_ab.log 2>&1; rc=$?
  tail -2 $OUT/t_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for st in ${STREAMS:-1 3}; do
  SKIP_TESTS=1 ROUNDS=${ROUNDS:-2} BENCH_ARGS="--streams $st ${BENCH_ARGS:-}" bash scripts/env_ab.sh || exit $?
done
