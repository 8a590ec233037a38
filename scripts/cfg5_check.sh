#!/bin/bash
# Config 5 (5M Gaussians, 1920x1080, SH 3): bench line with the training legs (densify/prune
# active), a 1-stream stage breakdown, and rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload cfg5_5m_1920x1080 --no-cpu-baseline > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
rc=$?; echo "cfg5 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_cfg5.err; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench_cfg5.json'));print(d['value'], d['train_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --workload cfg5_5m_1920x1080 --streams 1 --no-extra-legs --no-cpu-baseline > $OUT/bench_cfg5_1s.json 2> $OUT/bench_cfg5_1s.err
rc=$?; echo "cfg5 1 stream rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/bench_cfg5_1s.err; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench_cfg5_1s.json'));print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --workload cfg5_5m_1920x1080 --steps 2 --warmup 1 --no-cpu-baseline --no-stage-timing --no-extra-legs > $OUT/prof_cfg5.log 2>&1
rc=$?; echo "rocprof cfg5 rc=$rc"; exit $rc
