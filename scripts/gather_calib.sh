#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the duplication's record-gather shape (scripts/gather_calib.hip,
# built in-tree beforehand: hipcc --offload-arch=gfx950 -O3 -o scripts/gather_calib
# scripts/gather_calib.hip).  Two PMC passes (FETCH_SIZE and WRITE_SIZE cannot share one),
# then a per-kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/gcal
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/gcal/f -o f -- ./scripts/gather_calib ${N:-3000000} > $OUT/gcal_f.log 2>&1 || { tail -5 $OUT/gcal_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/gcal/w -o w -- ./scripts/gather_calib ${N:-3000000} > $OUT/gcal_w.log 2>&1 || { tail -5 $OUT/gcal_w.log; exit 1; }
python3 - ${N:-3000000} <<'PY'
import csv, glob, sys, collections
n = int(sys.argv[1])
names = {"15, true": "linear64", "1, false": "gather16", "3, false": "gather32", "11, false": "gather48", "15, false": "gather64"}
for tag in ("f", "w"):
    for path in glob.glob(f"gpurun_out/gcal/{tag}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for row in csv.DictReader(open(path)):
            k = row.get("Kernel_Name", "")
            if "gather_kernel" not in k:
                continue
            key = next((v for s, v in names.items() if s in k), k[:40])
            acc[(key, row["Counter_Name"])].append(float(row["Counter_Value"]))
        for (key, cn), vals in sorted(acc.items()):
            # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB
            per = [1024.0 * v / n for v in vals]
            print(f"{key:9s} {cn:10s} bytes/record per launch: " + " ".join(f"{p:.1f}" for p in per))
PY
