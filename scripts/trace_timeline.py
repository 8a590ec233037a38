"""Compact per-step timeline of a rocprofv3 kernel trace: one line per dispatch of the last
step-sized window (start offset, duration, queue, kernel class), so the pipeline's fill / drain
and the host-issue gaps can be read off directly.

usage: python3 scripts/trace_timeline.py <trace dir> <dispatches per step | auto> [steps back]"""
import csv
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_overlap import klass  # noqa: E402

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if sys.argv[2] == "auto":  # steps start at the SH colour pre-pass (one per step)
    starts = [i for i, r in enumerate(rows) if "sh_precolor" in r["Kernel_Name"]]
    a = starts[-back]
    b = starts[-back + 1] if back > 1 else len(rows)
    sel = rows[a:b]
else:
    per = int(sys.argv[2])
    sel = rows[-per * back:-per * (back - 1)] if back > 1 else rows[-per:]
t0 = int(sel[0]["Start_Timestamp"])
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r[qkey] if qkey else '?':>3} "
          f"{klass(r['Kernel_Name']):14s} {r['Kernel_Name'][:60]}")
