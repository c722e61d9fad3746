#!/usr/bin/env python3
"""Per-launch means of the band-KKT kernel's counters over the `pmcs` passes of scripts/session.sh (scripts/bandbench.py)
(one counter group per rocprofv3 --pmc run) plus the kernel-trace mean duration.
usage: band_pmc_summary.py [gpurun_out/bandpmc] [header line]"""
import collections, csv, glob, os, sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bandpmc"
vals, durs = collections.defaultdict(list), []
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_band_kkt" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(d, "p*", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_band_kkt" in r["Kernel_Name"]:
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print("# rocprofv3 --pmc passes over scripts/bandbench.py (65,536 x M = 10, band-KKT kernel, per-launch means)")
if len(sys.argv) > 2:
    print("# " + sys.argv[2])
print("# FETCH_SIZE/WRITE_SIZE in KB (FETCH_SIZE x2 on gfx950 for 16-B streaming reads).")
for k in sorted(vals):
    print(f"{k:24s} {sum(vals[k]) / len(vals[k]):.6g}")
if durs:
    print(f"kernel_trace_mean_ns     {sum(durs) / len(durs):.0f}  (n={len(durs)})")
if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
    fb = 2 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    wb = 1024 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    print(f"hbm_bytes_per_launch     {fb + wb:.4g}  (read {fb:.4g}, written {wb:.4g})")
