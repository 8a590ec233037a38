#!/bin/bash
# Round-2 measurement call: PMC passes at 6 views/step (headline workload) -> gpurun_out/pmc_r02.json,
# an isolated-stage bench at 1 stream, and the config-5 workload (5M, 1920x1080) bench line with
# its rocprofv3 kernel stats.  Each step has its own limit; the call stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${PMC:-1}" = "1" ]; then
  bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py $OUT/pmc $OUT/pmc_r02.json || exit $?
fi
timeout -k 10 300 python bench.py --streams 1 --no-extra-legs --no-cpu-baseline > $OUT/bench_1stream.json 2> $OUT/bench_1stream.err
rc=$?; echo "bench 1 stream rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_1stream.err; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench_1stream.json'));print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --workload cfg5_5m_1920x1080 --no-cpu-baseline ${CFG5_ARGS:-} > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
rc=$?; echo "bench cfg5 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_cfg5.err; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench_cfg5.json'));print(d['value'], d.get('train_step'), {k:v['avg_ms'] for k,v in d['kernels'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --workload cfg5_5m_1920x1080 --steps 2 --warmup 1 --no-cpu-baseline --no-stage-timing --no-extra-legs > $OUT/prof_cfg5.log 2>&1
rc=$?; echo "rocprof cfg5 rc=$rc"; exit $rc
