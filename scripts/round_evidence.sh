#!/bin/bash
# Everything the round's evidence needs, in one GPU call: PMC passes -> profiles summary, GPU tests,
# bench line, rocprofv3 kernel stats (scripts/refresh_profiles.sh), then smoke() and the 2-rank
# distributed rehearsal.  Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/refresh_profiles.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/dist_rehearsal.sh
