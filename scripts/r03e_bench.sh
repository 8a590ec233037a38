#!/bin/bash
# The bench line and the rocprofv3 kernel stats of the same command (bench defaults), after
# scripts/r03e_evidence.sh has produced profiles/pmc_r03e.json.  Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $OUT/b_evd.json 2> $OUT/b_evd.err || { tail -5 $OUT/b_evd.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/b_evd.json'));print('bench', d['value'], d['ms_per_step'], d['roofline'])"
rm -rf $OUT/prof_evd
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_evd -o run -- python3 bench.py > $OUT/b_prof_evd.json 2> $OUT/b_prof_evd.err || exit 4
find $OUT/prof_evd -name "*kernel_stats.csv"
