# A/B of radix-sort build variants (parity of the sort tests, sort micro-benchmark, bench.py)
# usage: LIBS="libgsr.so libgsr_noticket.so" bash scripts/kpt_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=sdp-gs_amd/gsr_amd
V=""
for k in ${LIBS:-libgsr.so}; do
  GSR_LIB_PATH=$L/$k timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -k "sort or scan" > gpurun_out/sortpar_$k.log 2>&1
  rc=$?; echo "parity $k rc=$rc $(tail -1 gpurun_out/sortpar_$k.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  V="$V GSR_LIB_PATH=$L/$k"
done
VARIANTS="$V" bash scripts/sort_ab.sh || exit $?
VARIANTS="$V $V" SKIP_TESTS=1 bash scripts/ab.sh
