#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/ttrace
timeout -k 10 300 python scripts/train_trace.py > gpurun_out/train_plain.log 2>&1; rc=$?; cat gpurun_out/train_plain.log | grep ms; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ttrace -o run -- python3 scripts/train_trace.py > gpurun_out/ttrace.log 2>&1; rc=$?; grep ms gpurun_out/ttrace.log; [ $rc -eq 0 ] || exit $rc
N=$(python3 -c "import glob,csv;f=glob.glob('gpurun_out/ttrace/**/*kernel_trace.csv',recursive=True)[0];print(sum(1 for _ in csv.DictReader(open(f)))//2)")
python3 scripts/trace_busy.py gpurun_out/ttrace $N
