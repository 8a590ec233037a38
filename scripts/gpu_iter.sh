#!/bin/bash
# One GPU iteration: selected GPU tests, then bench.py once per variant (alternating A/B rounds).
#   TESTS="tests/test_x.py ..."   test files (empty: skip the tests; "all": the whole -m gpu suite)
#   VARIANTS="A=1 A=0"            env assignments per bench run (comma joins several: "A=1,B=2")
#   ROUNDS=2                      how many times the variant list is repeated (alternating order)
#   BENCH_ARGS="--steps 10"       extra bench.py arguments (default: no CPU baseline, no extra legs)
# Output: gpurun_out/iter_*.json / .err, one summary line per bench run.  Stops at the first
# abnormal exit of any GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  T="$TESTS"; [ "$T" = "all" ] && T=tests
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v -s --timeout 1500 --timeout-method thread $T -m gpu > $OUT/iter_tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" $OUT/iter_tests.log | tail -3
  if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" $OUT/iter_tests.log | head -30; exit $rc; fi
fi
[ -z "${VARIANTS:-}" ] && [ -z "${BENCH:-}" ] && exit 0
i=0
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS:-NONE=1}; do
    i=$((i+1))
    env $(echo "$v" | tr ',' ' ') timeout -k 10 400 python bench.py --no-cpu-baseline --no-extra-legs ${BENCH_ARGS:-} > $OUT/iter_$i.json 2> $OUT/iter_$i.err
    rc=$?
    python3 - "$v" $OUT/iter_$i.json <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(sys.argv[1], "views/s", d["value"], "ms/step", round(d["ms_per_step"], 4),
          {n: round(k[n]["avg_ms"], 4) for n in k})
except Exception as e:
    print(sys.argv[1], "FAILED", e)
PY
    if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -5 $OUT/iter_$i.err; exit $rc; fi
  done
done
