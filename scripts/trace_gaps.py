"""GPU idle gaps of bench.py's steady-state steps from a rocprofv3 --sys-trace (csv), and for each
gap the host side of the kernel that ended it: when its launch call was made relative to the gap's
start (launched late by the host, or queued early and held by a dependency), and what the host
thread was doing just before.  Prints a small summary (the trace itself is too large to keep).

  python scripts/trace_gaps.py <rocprofv3 output dir> [steps to skip] [min gap us]
"""
import csv
import glob
import sys
from collections import Counter, defaultdict


def load(pattern):
    f = glob.glob(pattern, recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    return n.replace("gsr::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]


def main():
    d = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
    kt = load(f"{d}/**/*kernel_trace.csv")
    api = load(f"{d}/**/*hip_api_trace.csv") + load(f"{d}/**/*hsa_api_trace.csv")
    kern = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                    r.get("Correlation_Id")) for r in kt), key=lambda x: x[0])
    stream_of = {r.get("Correlation_Id"): (r.get("Stream_Id"), r.get("Queue_Id")) for r in kt}
    copies = load(f"{d}/**/*memory_copy_trace.csv")
    print(f"{len(copies)} memory copies")
    calls = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"],
                     r.get("Correlation_Id"), r.get("Thread_Id")) for r in api), key=lambda x: x[0])
    by_corr = {c[3]: c for c in calls}
    steps = [i for i, k in enumerate(kern) if "sh_precolor_kernel" in k[2]]
    print(f"{len(kern)} kernels, {len(calls)} HIP API calls, {len(steps)} steps")
    if kt and api:
        print("kernel columns:", list(kt[0].keys()))
        print("api columns:", list(api[0].keys()))
        print("sample kernel corr", kern[0][3], "api corr", calls[0][3], calls[0][2])
    gaps_by_next = defaultdict(list)
    span_tot = busy_tot = 0
    for a, b in list(zip(steps, steps[1:]))[skip:]:
        seg = kern[a:b]
        t_end = kern[b][0]
        busy, cs, ce = 0, seg[0][0], seg[0][1]
        for s, e, n, corr in seg[1:]:
            if s > ce:
                busy += ce - cs
                gap = (s - ce) / 1e3
                if gap >= min_gap:
                    launch = by_corr.get(corr)
                    if launch is None and not gaps_by_next:
                        near = [c for c in calls if abs(int(c[3] or 0) - int(corr or 0)) <= 2]
                        print("unmatched corr", corr, "nearby api ids:", [(c[3], c[2]) for c in near][:6])
                    rel = (launch[0] - ce) / 1e3 if launch else None  # launch time vs gap start
                    # the host calls of the launching thread in the gap window
                    prev = []
                    if launch:
                        prev = [c for c in calls if c[4] == launch[4] and ce - 200_000 <= c[0] < launch[0]]
                    slow = sorted(((c[1] - c[0]) / 1e3, c[2]) for c in prev)[-3:]
                    gaps_by_next[short(n)].append((gap, rel, slow))
                    if len(gaps_by_next[short(n)]) == 1:
                        prevk = max((k for k in seg if k[1] <= s), key=lambda k: k[1])
                        print(f"  example: {short(prevk[2])} on {stream_of.get(prevk[3])} ended, "
                              f"{short(n)} on {stream_of.get(corr)} started {gap:.1f} us later")
                        if launch:
                            lo = by_corr.get(prevk[3])
                            t_lo = lo[0] if lo else launch[0] - 2_000_000
                            between = [c[2] for c in calls if c[4] == launch[4] and t_lo < c[0] < launch[0]
                                       and ("Event" in c[2] or "Stream" in c[2] or "Memcpy" in c[2] or "Memset" in c[2])]
                            print("    host sync/stream calls between the two launches:", Counter(between).most_common(8))
                        cp = [c for c in copies if int(c["Start_Timestamp"]) < s and int(c["End_Timestamp"]) > ce - 50_000]
                        print("    copies overlapping the gap window:", [(c.get("Direction") or c.get("Kind"), (int(c["End_Timestamp"]) - int(c["Start_Timestamp"])) // 1000) for c in cp][:5])
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span_tot += t_end - seg[0][0]
        busy_tot += busy
    print(f"steady-state busy fraction {busy_tot / span_tot:.3f} over {span_tot / 1e3:.0f} us")
    for name, g in sorted(gaps_by_next.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        gs = [x[0] for x in g]
        rels = [x[1] for x in g if x[1] is not None]
        fn = [x for x in g if x[1] is not None]
        print(f"gap before {name}: n={len(g)} mean {sum(gs) / len(gs):.1f} us; launch call made "
              f"{(sum(rels) / len(rels)) if rels else float('nan'):+.1f} us after the gap began")
        cnt = Counter(s[1] for x in g for s in x[2])
        longest = sorted((s for x in g for s in x[2]), reverse=True)[:4]
        print("   host calls before the launch (longest):", [(round(t, 1), f) for t, f in longest],
              "| most frequent:", cnt.most_common(3))


if __name__ == "__main__":
    main()
