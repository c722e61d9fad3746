#!/usr/bin/env python3
"""Summarise gpurun_out/kpmc: mean counter value per dispatch of k_reduced_* per variant."""
import csv, glob, os, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kpmc"
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "k_reduced"
for var in sorted(os.listdir(root)):
    d = os.path.join(root, var)
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(list); dur = []
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if KERNEL not in row["Kernel_Name"]: continue
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            if KERNEL in row["Kernel_Name"]:
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    waves = sum(agg["SQ_WAVES"]) / max(len(agg["SQ_WAVES"]), 1)
    print(f"== {var}: dispatch {sorted(dur)[len(dur)//2] if dur else 0:.1f} us (median of {len(dur)})")
    for k in sorted(agg):
        v = sum(agg[k]) / len(agg[k])
        per = f"  per-wave {v / waves:.1f}" if waves and k.startswith("SQ_") and k != "SQ_WAVES" else ""
        print(f"   {k:26s} {v:14.4g}{per}")
