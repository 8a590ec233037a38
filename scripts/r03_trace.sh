#!/bin/bash
# Kernel-trace timeline of the headline step (GPU busy fraction, idle gaps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_r03 -o run -- python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs --no-stage-timing ${BENCH_ARGS:-} > gpurun_out/trace_r03.json 2> gpurun_out/trace_r03.err || exit $?
python3 scripts/trace_busy.py gpurun_out/trace_r03 ${NDISP:-1000}
