#!/bin/bash
# A/B of env-selected variants: runs the GPU tests once, then bench.py once per variant.
# usage: VARIANTS="GSR_BWD_GROUP=1 GSR_BWD_GROUP=4" bash scripts/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for v in ${VARIANTS:-NONE=1}; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab_$i.json 2> $OUT/ab_$i.err
  rc=$?
  python3 - "$v" $OUT/ab_$i.json <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    k = d["kernels"]
    print(sys.argv[1], "views/s", d["value"], {n: k[n]["avg_ms"] for n in k})
except Exception as e:
    print(sys.argv[1], "FAILED", e)
PY
  if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -3 $OUT/ab_$i.err; exit $rc; fi
done
