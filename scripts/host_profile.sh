#!/bin/bash
# Host-side (Python) cost of a bench step: cProfile of a short bench run, top functions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-stage-timing ${BENCH_ARGS:-} > gpurun_out/host_bench.json 2> gpurun_out/host_bench.err || exit $?
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/host.prof")
p.sort_stats("tottime").print_stats(25)
p.sort_stats("cumulative").print_stats(30)
PY
