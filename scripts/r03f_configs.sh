#!/bin/bash
# Config 5 (5M, 1920x1080) and config 2 (100k, 800x800) bench lines with the training legs, on the
# final build.  Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for w in cfg5_5m_1920x1080 cfg2_100k_800x800; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > $OUT/r03f_$w.json 2> $OUT/r03f_$w.err || { tail -5 $OUT/r03f_$w.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/r03f_$w.json'));print('$w', d['value'], d['ms_per_step'], {k:d[k]['value'] for k in ('train_step','reference_cadence','deterministic') if k in d})"
done
