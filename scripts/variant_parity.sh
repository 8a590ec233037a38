#!/bin/bash
# Parity of kernel variants before they are timed: the selected tests/test_fused_parity.py cases
# once per variant (env assignments, comma-joined as in gpu_iter.sh).
#   VARIANTS="GSR_BWD_PIPE=1 GSR_BWD_PIPE=2"   K="small_6views_3streams_multi or cfg3_1m_1008x756_multi"
# Output: gpurun_out/par_<n>.log; stops at the first failing or abnormal run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
K=${K:-small_6views_3streams_multi or cfg3_1m_1008x756_multi}
i=0
for v in ${VARIANTS:?set VARIANTS}; do
  i=$((i+1))
  env $(echo "$v" | tr ',' ' ') timeout -k 10 ${PAR_TIMEOUT:-400} python -u -m pytest -x -v -s --timeout $(( ${PAR_TIMEOUT:-400} - 20 )) --timeout-method thread tests/test_fused_parity.py -m gpu -k "$K" > $OUT/par_$i.log 2>&1
  rc=$?
  echo "$v parity rc=$rc: $(grep -E '[0-9]+ (passed|failed)' $OUT/par_$i.log | tail -1)"
  if [ $rc -ne 0 ]; then grep -E "^E |Error" $OUT/par_$i.log | head -20; exit $rc; fi
done
