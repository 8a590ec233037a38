#!/bin/bash
# Alternating bench runs of argument variants (separated by '|'), ROUNDS rounds, one process each.
# usage: ARGS_VARIANTS="--per-view|" ROUNDS=2 bash scripts/args_ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS='|' read -r -a VARS <<< "${ARGS_VARIANTS:-|}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VARS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs $v ${BENCH_ARGS:-} > $OUT/argab_$i.json 2> $OUT/argab_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench [$v] rc=$rc"; tail -5 $OUT/argab_$i.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/argab_$i.json'));print('round $r', '[$v]', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k in ('render_fwd','render_bwd','preprocess','duplicate','scan','depth_sort','tile_sort','preprocess_bwd')})"
  done
done
