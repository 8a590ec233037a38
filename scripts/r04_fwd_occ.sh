#!/bin/bash
# Round 4: forward-blend occupancy variants (lazy channel reads, 5/6 waves per SIMD; separate
# in-tree builds via GSR_LIB_PATH): parity, alternating bench runs, and one LDS-conflict PMC
# pass of the default build (preprocess after the swizzled zero-fill).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
VARIANTS="GSR_LIB_PATH=sdp-gs_amd/build_lazy6/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_lazy5/libgsr.so" bash scripts/variant_parity.sh || exit 1
rm -rf $OUT/pmc_lds
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_lds -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stage-timing --no-extra-legs > $OUT/pmc_lds.log 2>&1 || { tail -5 $OUT/pmc_lds.log; exit 1; }
python3 scripts/pmc_lds.py $OUT/pmc_lds | tee $OUT/pmc_lds.txt
VARIANTS="NONE=1 GSR_LIB_PATH=sdp-gs_amd/build_lazy5/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_lazy6/libgsr.so GSR_LIB_PATH=sdp-gs_amd/build_w5/libgsr.so" ROUNDS=2 bash scripts/gpu_iter.sh
