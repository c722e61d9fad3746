#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes (scripts/session.sh `pmcs` step: one counter group per run,
each under DIR/p<i>/) into per-kernel means per launch, one line per (kernel, counter).
FETCH_SIZE / WRITE_SIZE are in KB as rocprofv3 reports them; the gfx950 correction of the
HBM/rocprofv3 section of MI355X_MICROARCH.md (FETCH_SIZE counts each 64-B request once where
the fabric moves 128 B: x2) is applied in the derived HBM_BYTES line.
usage: pmc_fold.py DIR"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"^void ", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("(")[0]
        if name.startswith("__amd") or "elementwise" in name or "at::" in name:
            continue
        acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in acc})
for k in kern:
    short = k[-60:]
    vals = {c: sum(v) / len(v) for (kk, c), v in acc.items() if kk == k}
    n = max(len(v) for (kk, c), v in acc.items() if kk == k)
    for c in sorted(vals):
        print(f"{short:60s} {c:26s} {vals[c]:18.1f}  (n={n})")
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        print(f"{short:60s} {'HBM_BYTES(2xF+W)':26s} {1024.0 * (2.0 * vals['FETCH_SIZE'] + vals['WRITE_SIZE']):18.1f}")
