#!/bin/bash
# Round 6 evidence in GPU calls of at most ~15 minutes each (PART=pmc | bench | extra), outputs
# under gpurun_out/*_r06*; every GPU step has its own time limit and the script stops at the
# first abnormal exit.
#   pmc:   rocprofv3 --pmc passes of the headline bench -> gpurun_out/pmc_r06.json
#   bench: the default bench line (CPU baseline included), the rocprofv3 kernel-trace --stats of
#          the same command without CPU baseline / extra legs, smoke()
#   extra: the 2-rank launcher rehearsal (gloo ranks on the box's one GPU), the config-2 and
#          config-5 workloads, the train.py-cadence profile with per-stage GPU times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
case "${PART:?set PART=pmc|bench|extra}" in
pmc)
  rm -rf $OUT/pmc
  COUNTERS=profiles/counters_r05.txt bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py $OUT/pmc $OUT/pmc_r06.json || exit $?
  ;;
bench)
  timeout -k 10 600 python bench.py --pmc-file profiles/pmc_r06.json > $OUT/b_r06.json 2> $OUT/b_r06.err || { tail -5 $OUT/b_r06.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/b_r06.json'));print('bench', d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac'])"
  rm -rf $OUT/prof_r06
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r06 -o run -- python3 bench.py --no-cpu-baseline --no-extra-legs --pmc-file profiles/pmc_r06.json > $OUT/b_prof_r06.json 2> $OUT/b_prof_r06.err || exit 4
  find $OUT/prof_r06 -name "*kernel_stats.csv"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_r06.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $OUT/smoke_r06.log; exit $rc
  ;;
extra)
  GSR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/dist2_r06.json 2> $OUT/dist2_r06.err; rc=$?
  echo "dist2 rc=$rc"; cut -c1-300 $OUT/dist2_r06.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --workload cfg2_100k_800x800 --no-cpu-baseline --no-extra-legs > $OUT/cfg2_r06.json 2> $OUT/cfg2_r06.err || exit 5
  timeout -k 10 400 python bench.py --workload cfg5_5m_1920x1080 --no-cpu-baseline --no-extra-legs > $OUT/cfg5_r06.json 2> $OUT/cfg5_r06.err || exit 6
  timeout -k 10 300 python -u scripts/cadence_profile.py --stages > $OUT/cadence_r06.json 2> $OUT/cadence_r06.err || exit 7
  cat $OUT/cadence_r06.json
  ;;
esac
