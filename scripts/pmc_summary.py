#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one directory per pass) into profiles/pmc_rNN.json.

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads exactly half of the bytes of a
wide coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.  Both are
per-dispatch averages.  Counter values are averages over the dispatches of each kernel."""
import collections
import csv
import glob
import json
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_r01.json"
workload = sys.argv[3] if len(sys.argv) > 3 else "llff_1m_1008x756"
STAGE = {"preprocess_kernel": "preprocess", "duplicate_kernel": "duplicate",
         "tile_ranges_kernel": "ranges", "render_fwd_kernel": "render_fwd",
         "render_fwd_blk_kernel": "render_fwd",
         "render_bwd_kernel": "render_bwd", "preprocess_bwd_kernel": "preprocess_bwd",
         # multi-view calls: several views per launch
         "render_bwd_views_kernel": "render_bwd", "render_fwd_blk_views_kernel": "render_fwd",
         "preprocess_bwd_views_kernel": "preprocess_bwd",
         # batched binning of the multi-view forward
         "preprocess_views_kernel": "preprocess", "duplicate_views_kernel": "duplicate",
         "tile_ranges_views_kernel": "ranges", "radix_totals_views_kernel": "radix_totals",
         "radix_onesweep_views_kernel": "radix_onesweep", "scan_reduce_views_kernel": "scan_reduce",
         "scan_final_views_kernel": "scan_final", "scan_parts_views_kernel": "scan_parts",
         "sum_parts_views_kernel": "sum_parts", "tile_schedule_views_kernel": "schedule",
         "radix_totals_kernel": "radix_totals", "radix_onesweep_kernel": "radix_onesweep",
         "scan_reduce_kernel": "scan_reduce", "scan_final_kernel": "scan_final",
         "scan_parts_kernel": "scan_parts", "sh_precolor_kernel": "sh_precolor",
         "sh_flush_kernel": "sh_flush"}
agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for f in sorted(glob.glob(f"{src}/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        if not m or m.group(1) not in STAGE:
            continue
        name = STAGE[m.group(1)]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[name] = {"vgpr": int(r["VGPR_Count"]), "lds_bytes": int(r["LDS_Block_Size"]),
                      "workgroup": int(r["Workgroup_Size"])}
kernels = {}
for name, d in agg.items():
    c = {k: sum(v) / len(v) for k, v in d.items()}
    k = {"counters": {n: round(v, 1) for n, v in sorted(c.items())}, **meta.get(name, {})}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        k["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        k["valu_active_per_wave_cycle"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        k["wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU", 0) > 0:
        # lanes with EXEC on per VALU issue cycle, of 64 (both counters in the same units):
        # counts every enabled lane, not only the ones doing useful work
        k["valu_exec_lane_frac"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
    if "SQ_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"] > 0:
        k["sq_busy_frac"] = round(c["SQ_BUSY_CYCLES"] / c["GRBM_GUI_ACTIVE"], 4)
    kernels[name] = k
json.dump({"workload": workload, "source": src, "kernels": kernels}, open(out, "w"), indent=1)
for n, k in kernels.items():
    print(n, {x: k[x] for x in k if x != "counters"})
    print("   ", k["counters"])
