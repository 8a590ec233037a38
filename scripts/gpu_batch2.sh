#!/bin/bash
# round-6 GPU batch: parity of the band-cut build (binning + blend masks), then an A/B of the
# library variants (base = before, band = backward masks, band2 = + forward masks, band3 = + binning)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_index_parity.py tests/test_batched_binning.py tests/test_gpu_parity.py "tests/test_fused_parity.py::test_benchmarked_path_matches_oracle" -m gpu -k "not cfg5 and not cfg3_1m_1008x756]" > $OUT/t_band.log 2>&1; rc=$?
tail -3 $OUT/t_band.log; [ $rc -eq 0 ] || exit $rc
LIBS="sdp-gs_amd/gsr_amd/libgsr_base.so|sdp-gs_amd/gsr_amd/libgsr_band.so|sdp-gs_amd/gsr_amd/libgsr_band2.so|sdp-gs_amd/gsr_amd/libgsr_band3.so" STAGES=render_bwd,render_fwd,preprocess,duplicate,tile_sort ROUNDS=2 bash scripts/lib_ab.sh
