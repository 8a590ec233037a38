#!/bin/bash
# GPU suite (optional), then alternating 1-stream / 3-stream bench runs of env-selected variants.
# usage: VARIANTS="GSR_BWD_MFMA=0 GSR_BWD_MFMA=1" [SKIP_TESTS=1] [BENCH_ARGS=...] bash scripts/env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in ${VARIANTS:-NONE=1}; do
    i=$((i+1))
    env $v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs ${BENCH_ARGS:-} > $OUT/envab_$i.json 2> $OUT/envab_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench [$v] rc=$rc"; tail -3 $OUT/envab_$i.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/envab_$i.json'));print('round $r', '$v', d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k in ('render_fwd','render_bwd','preprocess','duplicate','scan','depth_sort','tile_sort','preprocess_bwd')})"
  done
done
