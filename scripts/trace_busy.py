"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals over the span of the
last N dispatches (the timed steps), and the biggest idle gaps."""
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50])
               for r in csv.DictReader(open(f))), key=lambda x: x[0])
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
rows = rows[-n:]
t0, t1 = rows[0][0], max(e for _, e, _ in rows)
busy, cur_s, cur_e, gaps = 0, rows[0][0], rows[0][1], []
for s, e, name in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, name))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / (t1 - t0):.1f}%), "
      f"{len(gaps)} gaps, idle {(t1 - t0 - busy) / 1e3:.1f} us")
for g, name in sorted(gaps, reverse=True)[:8]:
    print(f"  gap {g / 1e3:.1f} us before {name}")
