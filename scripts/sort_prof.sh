#!/bin/bash
# rocprofv3 kernel stats of scripts/sort_bench.py (radix sort micro-benchmark)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/sortprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sortprof -o run -- python3 scripts/sort_bench.py > gpurun_out/sortprof.log 2>&1
rc=$?
grep "ms/sort" gpurun_out/sortprof.log
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/sortprof/**/run_kernel_stats.csv', recursive=True)
for r in list(csv.DictReader(open(f[0])))[:8]:
    print(f"calls={r['Calls']:>5} avg={float(r['AverageNs'])/1000:8.2f}us min={float(r['MinNs'])/1000:8.2f} max={float(r['MaxNs'])/1000:8.2f} {r['Name'][:60]}")
PY
exit $rc
