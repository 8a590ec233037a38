#!/bin/bash
# Round-3 GPU iteration: full GPU suite, default bench, the 2-rank launcher rehearsal (gloo on one
# GPU), a rocprofv3 kernel-stats pass of the bench.  Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > gpurun_out/t_r03.log 2>&1; rc=$?
tail -15 gpurun_out/t_r03.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/b_r03.json 2> gpurun_out/b_r03.err || { tail -20 gpurun_out/b_r03.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/b_r03.json'));print(d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['config']['num_rendered_mean'], d['config']['instances_mean'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, {k:d[k].get('value') for k in ('train_step','reference_cadence','reference_api','deterministic') if k in d})"
GSR_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dist2_r03.json 2> gpurun_out/dist2_r03.err; rc=$?
echo "dist2 rc=$rc"; cut -c1-400 gpurun_out/dist2_r03.json; tail -3 gpurun_out/dist2_r03.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-extra-legs > gpurun_out/b_prof_r03.json 2> gpurun_out/b_prof_r03.err || exit 4
  find gpurun_out/prof_r03 -name "*kernel_stats.csv" | head -2
fi
