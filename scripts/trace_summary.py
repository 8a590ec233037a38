"""Per (kernel, grid, workgroup) call counts and mean durations from a rocprofv3 kernel-trace CSV."""
import collections, csv, glob, sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    name = r.get("Kernel_Name", "").replace("gsr::(anonymous namespace)::", "").replace("void ", "")
    if "(" in name:
        name = name[:name.index("(")]
    key = (name[:60], r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", "?"))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/tot*100:6.2f}% n={len(v):4d} mean={sum(v)/len(v):8.2f}us grid={k[1]:>9s} wg={k[2]:>5s} {k[0]}")
