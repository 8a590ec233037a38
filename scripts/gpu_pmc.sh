#!/bin/bash
# PMC collection (separate passes, no tracing domains): per-kernel counters for the roofline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 -i ${COUNTERS:-profiles/counters_r05.txt} --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py --steps 1 --warmup 1 --views-per-gpu 6 --no-cpu-baseline --no-stage-timing --no-extra-legs ${BENCH_ARGS:-} > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -5 $OUT/pmc.log; find $OUT/pmc -name "*.csv" | head -20
