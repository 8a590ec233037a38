#!/bin/bash
# Round 4 forward-blend batch: blend statistics (instrumented build), the record-gather FETCH_SIZE
# calibration, parity of the GSR_FWD_FAST variants, then alternating bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
GSR_LIB_PATH=$PWD/sdp-gs_amd/build_stats/libgsr.so timeout -k 10 300 python scripts/blend_stats.py > $OUT/blend_stats_r04.txt 2>&1 || { tail -5 $OUT/blend_stats_r04.txt; exit 1; }
tail -6 $OUT/blend_stats_r04.txt
bash scripts/gather_calib.sh > $OUT/gather_calib_r04.txt 2>&1 || { tail -5 $OUT/gather_calib_r04.txt; exit 1; }
cat $OUT/gather_calib_r04.txt
VARIANTS="GSR_FWD_FAST=1 GSR_FWD_FAST=3" K="small_6views_3streams_multi or cfg3_1m_1008x756_multi or cfg5_5m_1920x1080_multi" PAR_TIMEOUT=900 bash scripts/variant_parity.sh || exit 1
VARIANTS="GSR_FWD_FAST=0 GSR_FWD_FAST=1 GSR_FWD_FAST=2 GSR_FWD_FAST=3" ROUNDS=2 bash scripts/gpu_iter.sh
