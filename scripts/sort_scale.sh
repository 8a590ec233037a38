#!/bin/bash
# Sort micro-benchmark at the headline and config-5 sizes (kernel trace split by grid size), and the
# config-5 bench at one stream (isolated stage times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/sortscale
SORT_LARGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sortscale -o run -- python3 scripts/sort_bench.py > gpurun_out/sortscale.log 2>&1
rc=$?; grep "ms/sort" gpurun_out/sortscale.log; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/sortscale/**/run_kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r['Kernel_Name'].split('(')[0][-40:]
    agg[(name, r['Grid_Size_X'] if 'Grid_Size_X' in r else r.get('Grid_Size',''), r.get('Workgroup_Size_X', ''))].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in sorted(agg.items()):
    v = sorted(v)
    print(k, len(v), 'median us', v[len(v)//2] / 1000)
PY
[ "${CFG5:-1}" = "1" ] || exit 0
timeout -k 10 300 python bench.py --workload cfg5_5m_1920x1080 --streams 1 --no-extra-legs --no-cpu-baseline > gpurun_out/bench_cfg5_1s.json 2> gpurun_out/bench_cfg5_1s.err
rc=$?; echo "cfg5 1 stream rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_cfg5_1s.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_cfg5_1s.json'));print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
