#!/bin/bash
# Alternating bench runs of environment variants (separated by '|', each a space-separated list
# of VAR=value), ROUNDS rounds, one process each; prints value and ms/step per run.
# usage: ENV_VARIANTS="GSR_VIEWS_BATCHED=0|GSR_VIEWS_BATCHED=1" ROUNDS=2 bash scripts/env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS='|' read -r -a VARS <<< "${ENV_VARIANTS:-X=0}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VARS[@]}"; do
    i=$((i+1))
    env $v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs --no-stage-timing ${BENCH_ARGS:-} > $OUT/envab_$i.json 2> $OUT/envab_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench [$v] rc=$rc"; tail -5 $OUT/envab_$i.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/envab_$i.json'));print('round $r', '[$v]', d['value'], d['ms_per_step'])"
  done
done
