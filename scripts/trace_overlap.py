"""Overlap breakdown of a rocprofv3 kernel trace over the last N dispatches (the timed steps):
for every instant, which kernel classes are running.  Reports the fraction of the span during
which a blend (render_fwd / render_bwd) runs, and for the rest which classes run alone -- the
wall time the binning / preprocessing chain is NOT hidden behind a blend.

usage: python3 scripts/trace_overlap.py <trace dir> [N dispatches]"""
import collections
import csv
import glob
import sys

CLASSES = [("render_bwd", "render_bwd"), ("render_fwd", "render_fwd"),
           ("preprocess_bwd", "preprocess_bwd"), ("preprocess_kernel", "preprocess"),
           ("radix_onesweep", "sort"), ("radix_totals", "sort"), ("duplicate", "duplicate"),
           ("scan_", "scan"), ("sum_parts", "scan"), ("tile_ranges", "ranges"),
           ("tile_schedule", "ranges"), ("sh_precolor", "sh_prepass"), ("sh_flush", "sh_flush")]


def klass(name):
    for key, c in CLASSES:
        if key in name:
            return c
    return "other"


def main():
    f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"]))
                   for r in csv.DictReader(open(f))), key=lambda x: x[0])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
    rows = rows[-n:]
    ev = []
    for s, e, c in rows:
        ev.append((s, 1, c))
        ev.append((e, -1, c))
    ev.sort()
    active = collections.Counter()
    t_prev = ev[0][0]
    span = ev[-1][0] - ev[0][0]
    state_time = collections.Counter()
    for t, d, c in ev:
        dt = t - t_prev
        if dt > 0:
            running = frozenset(k for k, v in active.items() if v > 0)
            if not running:
                state_time["idle"] += dt
            elif "render_bwd" in running or "render_fwd" in running:
                state_time["blend running"] += dt
            else:
                state_time["no blend: " + "+".join(sorted(running))] += dt
        active[c] += d
        t_prev = t
    print(f"span {span / 1e3:.1f} us over {len(rows)} dispatches")
    for k, v in state_time.most_common(20):
        print(f"  {100 * v / span:5.1f}%  {v / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
