#!/bin/bash
# A round's evidence in one GPU call, tagged (usage: TAG=r04 bash scripts/evidence.sh):
#   PMC passes -> profiles/pmc_$TAG.json (bench's roofline.traffic and VALU figures),
#   the GPU suite, the bench line, rocprofv3 kernel stats of the same bench command, smoke(),
#   the 2-rank launcher rehearsal (gloo on one GPU).
# Outputs under gpurun_out/*_$TAG*; stops at the first abnormal exit.
set -u
TAG=${TAG:?set TAG, e.g. TAG=r04}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${SKIP_PMC:-0}" != "1" ]; then
  rm -rf $OUT/pmc
  bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py $OUT/pmc profiles/pmc_$TAG.json && cp profiles/pmc_$TAG.json $OUT/pmc_$TAG.json || exit $?
fi
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -v -s --timeout 1500 --timeout-method thread tests -m gpu > $OUT/t_$TAG.log 2>&1; rc=$?
  tail -3 $OUT/t_$TAG.log; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 600 python bench.py > $OUT/b_$TAG.json 2> $OUT/b_$TAG.err || { tail -5 $OUT/b_$TAG.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/b_$TAG.json'));print('bench', d['value'], d['roofline'])"
rm -rf $OUT/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --no-extra-legs > $OUT/b_prof_$TAG.json 2> $OUT/b_prof_$TAG.err || exit 4
find $OUT/prof_$TAG -name "*kernel_stats.csv"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
GSR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/dist2_$TAG.json 2> $OUT/dist2_$TAG.err; rc=$?
echo "dist2 rc=$rc"; cut -c1-300 $OUT/dist2_$TAG.json; exit $rc
