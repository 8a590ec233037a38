#!/bin/bash
# PMC passes (profiles/counters_r01.txt, one rocprofv3 run per line) of the headline bench for
# several library builds: LIBS="default|sdp-gs_amd/gsr_amd/libgsr_x.so" (GSR_LIB_PATH values;
# "default" = the in-tree libgsr.so).  Summaries: gpurun_out/pmc_ab_<i>.json (scripts/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS='|' read -r -a VARS <<< "${LIBS:-default}"
i=0
for v in "${VARS[@]}"; do
  i=$((i+1))
  if [ "$v" = "default" ]; then unset GSR_LIB_PATH; else export GSR_LIB_PATH="$v"; fi
  rm -rf $OUT/pmc_ab_$i
  timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 -i ${COUNTERS:-profiles/counters_r05.txt} --output-format csv -d $OUT/pmc_ab_$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --views-per-gpu 6 --no-cpu-baseline --no-stage-timing --no-extra-legs ${BENCH_ARGS:-} > $OUT/pmc_ab_$i.log 2>&1
  rc=$?; echo "[$v] pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_ab_$i.log; exit $rc; }
  python3 scripts/pmc_summary.py $OUT/pmc_ab_$i $OUT/pmc_ab_$i.json | grep -E "^render_bwd|^render_fwd"
done
