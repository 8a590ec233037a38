#!/bin/bash
# Round 4: the f64 parity test, then --view-chunks A/B (alternating), then a kernel trace of the
# 1- and 2-chunk steps for the timeline (scripts/trace_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -f $OUT/f64_stats.jsonl
timeout -k 10 900 python -u -m pytest -v -s --timeout 880 --timeout-method thread tests/test_f64_parity.py tests/test_parallel_gpu.py -m gpu > $OUT/t_f64.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/t_f64.log | tail -2; [ $rc -le 1 ] || exit $rc
ARGSETS="--view-chunks 1|--view-chunks 2|--view-chunks 3" ROUNDS=2 STEPS=20 bash scripts/args_ab.sh || exit 1
for c in 1 2; do
  rm -rf $OUT/trace_c$c
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_c$c -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-stage-timing --no-extra-legs --view-chunks $c > $OUT/trace_c$c.log 2>&1 || exit 4
  python3 scripts/trace_timeline.py $OUT/trace_c$c auto 2 > $OUT/timeline_c$c.txt 2>&1
  python3 scripts/trace_busy.py $OUT/trace_c$c > $OUT/busy_c$c.txt 2>&1
  tail -3 $OUT/busy_c$c.txt
done
