#!/bin/bash
# round-6 GPU batch: parity suites touched this round, the cadence profile, a quick bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_f64_parity.py tests/test_gpu_parity.py tests/test_index_parity.py tests/test_backstop.py -m gpu > $OUT/t_new2.log 2>&1; rc=$?
tail -3 $OUT/t_new2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/cadence_profile.py --stages > $OUT/cadence.json 2> $OUT/cadence.err; rc=$?
cat $OUT/cadence.json; tail -3 $OUT/cadence.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b1.json 2> $OUT/b1.err; rc=$?
tail -3 $OUT/b1.err; python3 -c "import json;d=json.load(open('$OUT/b1.json'));print(d['value'], d['roofline']['avg_ms'], {k:d[k].get('value') for k in ('train_step','reference_cadence','reference_api','deterministic') if k in d})"
exit $rc
