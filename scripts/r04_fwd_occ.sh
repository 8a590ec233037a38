#!/bin/bash
# Round 4: forward-blend occupancy variants (lazy channel reads, 5/6 waves per SIMD) and the
# duplication's packed row ranges (separate in-tree builds via GSR_LIB_PATH): index and fused
# parity, alternating bench runs, and one LDS-conflict PMC pass of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 480 --timeout-method thread tests/test_index_parity.py tests/test_batched_binning.py tests/test_deterministic.py -m gpu > $OUT/t_rowpack.log 2>&1
rc=$?; tail -2 $OUT/t_rowpack.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="NONE=1 GSR_LIB_PATH=sdp-gs_amd/build_lazy6/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_lazy5/libgsr.so" bash scripts/variant_parity.sh || exit 1
rm -rf $OUT/pmc_lds
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_lds -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stage-timing --no-extra-legs > $OUT/pmc_lds.log 2>&1 || { tail -5 $OUT/pmc_lds.log; exit 1; }
python3 scripts/pmc_lds.py $OUT/pmc_lds | tee $OUT/pmc_lds.txt
VARIANTS="NONE=1 GSR_LIB_PATH=sdp-gs_amd/build_norp/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_lazy5/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_lazy6/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_w5/libgsr.so" ROUNDS=2 bash scripts/gpu_iter.sh
