#!/bin/bash
# rocprofv3 kernel trace of a short bench run; per (kernel, grid) durations via scripts/trace_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stage-timing --streams ${STREAMS:-1} ${BENCH_ARGS:-} > gpurun_out/trace.log 2>&1 || exit $?
python3 scripts/trace_summary.py gpurun_out/trace
