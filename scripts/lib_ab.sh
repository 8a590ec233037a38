#!/bin/bash
# Alternating bench runs of library builds (GSR_LIB_PATH values separated by '|'; "default" = the
# in-tree libgsr.so; an entry containing '=' is a space-separated list of VAR=value instead), ROUNDS rounds; prints value, ms/step and the named stages' avg ms.
# usage: LIBS="default|sdp-gs_amd/gsr_amd/libgsr_x.so" STAGES="preprocess_bwd" bash scripts/lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS='|' read -r -a VARS <<< "${LIBS:-default}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VARS[@]}"; do
    i=$((i+1))
    if [ "$v" = "default" ]; then E="X=0"; elif [[ "$v" == *=* ]]; then E="$v"; else E="GSR_LIB_PATH=$v"; fi
    env $E timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extra-legs ${BENCH_ARGS:-} > $OUT/libab_$i.json 2> $OUT/libab_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench [$v] rc=$rc"; tail -5 $OUT/libab_$i.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/libab_$i.json'));print('round $r', '[$v]', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k in '${STAGES:-render_bwd}'.split(',')})"
  done
done
