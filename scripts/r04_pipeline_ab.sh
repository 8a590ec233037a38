#!/bin/bash
# Round 4 step-pipeline batch: parity of the new issue orders / kernels, then alternating bench
# runs of the defaults against each change switched off (or the candidate switched on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 480 --timeout-method thread tests/test_batched_binning.py tests/test_deterministic.py tests/test_render.py tests/test_parallel_gpu.py -m gpu > $OUT/t_pipe.log 2>&1
rc=$?; tail -2 $OUT/t_pipe.log; [ $rc -eq 0 ] || exit $rc
GSR_PRE_VIEWS_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_batched_binning.py -m gpu > $OUT/t_presplit.log 2>&1
rc=$?; tail -1 $OUT/t_presplit.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="NONE=1 GSR_PRE_VIEWS_SPLIT=1" bash scripts/variant_parity.sh || exit 1
VARIANTS="${AB:-NONE=1 GSR_VIEWS_BIN_FIRST=0 GSR_PRECOLOR_SPLIT=0 GSR_PRE_VIEWS_SPLIT=1}" ROUNDS=${ROUNDS:-3} bash scripts/gpu_iter.sh
