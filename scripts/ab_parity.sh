#!/bin/bash
# One GPU call for a kernel change: the full GPU suite (incl. the fused-path oracle parity) on the
# in-tree build, then alternating bench runs of the baseline build (LIB_BASE) and the new one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=sdp-gs_amd/gsr_amd
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-libgsr_base.so libgsr.so}; do
    GSR_LIB_PATH=$L/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs ${BENCH_ARGS:-} > $OUT/ab_$lib.json 2> $OUT/ab_$lib.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; tail -3 $OUT/ab_$lib.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/ab_$lib.json'));print('round $r', '$lib', d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k in ('render_fwd','render_bwd','preprocess','duplicate','scan','depth_sort','tile_sort')})"
  done
done
