#!/bin/bash
# GPU suite (default atomics backward), then the rows-layout parity subset (GSR_BWD_ROWS=1);
# stops at the first failure of either.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/t_def.log 2>&1; rc=$?
tail -3 $OUT/t_def.log; [ $rc -eq 0 ] || exit $rc
GSR_BWD_ROWS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backstop.py tests/test_gpu_parity.py tests/test_deterministic.py tests/test_render.py tests/test_index_parity.py tests/test_configs.py "tests/test_fused_parity.py::test_benchmarked_path_matches_oracle" -k "not cfg5" -m gpu > $OUT/t_rows.log 2>&1; rc=$?
tail -3 $OUT/t_rows.log; exit $rc
