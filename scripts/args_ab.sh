#!/bin/bash
# A/B of bench.py argument sets, alternated ROUNDS times on one box (run-to-run spread between
# boxes is a few %, so compare only within one call).
# usage: ARGSETS="--streams 2|--streams 2 --no-defer-sh" ROUNDS=3 bash scripts/args_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS='|' read -ra SETS <<< "${ARGSETS:---streams 2}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in "${!SETS[@]}"; do
    a="${SETS[$i]}"
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-stage-timing $a > gpurun_out/abargs_$i.json 2> gpurun_out/abargs_$i.err || { echo "bench rc=$? for [$a]"; tail -3 gpurun_out/abargs_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abargs_$i.json').read().strip().splitlines()[-1]); print('round $r', '[$a]', d['value'])"
  done
done
