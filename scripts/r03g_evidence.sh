#!/bin/bash
# Round-3 evidence (final build: batched binning, LDS-staged duplication) in one GPU call: PMC passes -> profiles/pmc_r03g.json (bench's roofline.traffic
# and VALU figures), GPU suite, bench line, rocprofv3 kernel stats of the same command, smoke(),
# the 2-rank launcher rehearsal (gloo on one GPU).  Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/pmc
bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py $OUT/pmc profiles/pmc_r03g.json && cp profiles/pmc_r03g.json $OUT/pmc_r03g.json || exit $?
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/t_evd.log 2>&1; rc=$?
tail -3 $OUT/t_evd.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/b_evd.json 2> $OUT/b_evd.err || { tail -5 $OUT/b_evd.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/b_evd.json'));print('bench', d['value'], d['roofline'])"
rm -rf $OUT/prof_evd
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_evd -o run -- python3 bench.py > $OUT/b_prof_evd.json 2> $OUT/b_prof_evd.err || exit 4
find $OUT/prof_evd -name "*kernel_stats.csv"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_evd.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke_evd.log; [ $rc -eq 0 ] || exit $rc
GSR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/dist2_evd.json 2> $OUT/dist2_evd.err; rc=$?
echo "dist2 rc=$rc"; cut -c1-300 $OUT/dist2_evd.json; exit $rc
