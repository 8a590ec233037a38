# A/B of library builds: GPU test suite against each build, then bench.py per build
# usage: LIBS="libgsr.so libgsr_x.so" [TESTS="tests -m gpu"] bash scripts/lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=sdp-gs_amd/gsr_amd
V=""
for k in ${LIBS:-libgsr.so}; do
  GSR_LIB_PATH=$L/$k timeout -k 10 900 python -m pytest ${TESTS:-tests -m gpu} -q -x > gpurun_out/tests_$k.log 2>&1
  rc=$?; echo "tests $k rc=$rc $(tail -1 gpurun_out/tests_$k.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  V="$V GSR_LIB_PATH=$L/$k"
done
VARIANTS="$V $V" SKIP_TESTS=1 bash scripts/ab.sh
