#!/bin/bash
# A/B of sort variants with the sort micro-benchmark under rocprofv3.
# VARIANTS="GSR_SORT_X=0 GSR_SORT_X=8,GSR_LIB_PATH=..." (comma-separated env assignments per variant)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-NONE=1}; do
  echo "== $v"
  env ${v//,/ } bash scripts/sort_prof.sh | grep -v "calls=  19\|calls=    2" || exit $?
done
