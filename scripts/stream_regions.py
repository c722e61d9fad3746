#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `bench.py` (default --streams 2) into its two timed
kinds of headline launches and summarise each:
  overlapped    launches that overlap another launch of the kernel in time (the headline
                region: consecutive batches alternating between two streams);
  back_to_back  launches that overlap none (the one-stream pass the roofline is timed on,
                the warm-up and the per-launch side line).
For each: launches, mean / median kernel duration, and the span per launch of the
longest run of consecutive launches of that kind (what the region's events measure).
    python3 scripts/stream_regions.py TRACE_CSV [KERNEL_SUBSTRING]"""
import csv, json, statistics as st, sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_lane_uniform<10"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(path)) if name in r["Kernel_Name"])
kind = []
for i, (s, e) in enumerate(ks):
    prev_e = ks[i - 1][1] if i else -1
    next_s = ks[i + 1][0] if i + 1 < len(ks) else 1 << 62
    kind.append("overlapped" if (prev_e > s or next_s < e) else "back_to_back")
out = {"trace": path, "kernel": name, "launches": len(ks)}
for k in ("overlapped", "back_to_back"):
    d = [(e - s) / 1e3 for (s, e), kk in zip(ks, kind) if kk == k]
    runs, cur = [], []
    for (s, e), kk in zip(ks, kind):
        if kk == k:
            cur.append((s, e))
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    best = max(runs, key=len) if runs else []
    span = (max(e for _, e in best) - best[0][0]) / 1e3 / len(best) if best else None
    out[k] = {"launches": len(d), "mean_us": st.mean(d) if d else None, "median_us": st.median(d) if d else None,
              "longest_run": len(best), "span_us_per_launch_of_longest_run": span}
print(json.dumps(out, indent=1))
