#!/bin/bash
# Rows layout (GSR_BWD_ROWS=1) parity subset on the GPU, then alternating 1- and 3-stream bench
# runs: atomics / rows / the DIAG=2 build (flush as plain stores: what the atomics cost).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
GSR_BWD_ROWS=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_deterministic.py tests/test_render.py tests/test_index_parity.py tests/test_backstop.py tests/test_configs.py "tests/test_fused_parity.py::test_benchmarked_path_matches_oracle" -k "not cfg5" -m gpu > $OUT/t_rows.log 2>&1; rc=$?
tail -3 $OUT/t_rows.log; [ $rc -le 1 ] || exit $rc
L=sdp-gs_amd/gsr_amd
for st in 1 3; do
  VARIANTS="GSR_BWD_ROWS=0 GSR_BWD_ROWS=1 GSR_LIB_PATH=$L/libgsr_diag2.so" SKIP_TESTS=1 ROUNDS=2 BENCH_ARGS="--streams $st" bash scripts/env_ab.sh || exit $?
done
