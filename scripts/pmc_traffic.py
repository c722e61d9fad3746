#!/usr/bin/env python3
"""Fold the PMC passes of scripts/gpu_profile.sh into profiles/pmc_traffic.json.

HBM bytes per launch of the dominant kernel, corrected as MI355X_MICROARCH.md's
HBM section prescribes for gfx950:
  FETCH_SIZE (KB) reports half the bytes of a wide coalesced read -> x 2
  WRITE_SIZE (KB) is exact for 16-B-per-lane streaming stores
Each counter comes from its own --pmc pass (they cannot share one).

usage: pmc_traffic.py [gpurun_out/pmc] [key]      key e.g. B65536_M10_reduced_sets4
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(pmc_dir, kernel_substr):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(pmc_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    pmc_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    key = sys.argv[2] if len(sys.argv) > 2 else "B65536_M10_reduced_sets4"
    if "reduced" in key:  # uniform even M: the lane-per-trajectory kernel; odd M: the lane-pair one
        M = int(key.split("_M")[1].split("_")[0])
        kernel = "k_lane_uniform" if M % 2 == 0 else "k_reduced_uniform"
    else:
        kernel = "k_dense_kkt"
    mean, n = per_dispatch(pmc_dir, kernel)
    if "FETCH_SIZE" not in mean or "WRITE_SIZE" not in mean:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE for {kernel} under {pmc_dir}")
    fetch = mean["FETCH_SIZE"] * 1024.0 * 2.0
    write = mean["WRITE_SIZE"] * 1024.0
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(out_path))
    except (OSError, ValueError):
        d = {}
    d[key] = {
        "kernel": kernel,
        "hbm_bytes_per_launch": fetch + write,
        "read_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "raw_FETCH_SIZE_KB": mean["FETCH_SIZE"],
        "raw_WRITE_SIZE_KB": mean["WRITE_SIZE"],
        "dispatches": {"FETCH_SIZE": n["FETCH_SIZE"], "WRITE_SIZE": n["WRITE_SIZE"]},
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; KB = 1024 B",
        "other_counters": {k: v for k, v in mean.items() if k not in ("FETCH_SIZE", "WRITE_SIZE")},
    }
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: d[key]["hbm_bytes_per_launch"]}))


if __name__ == "__main__":
    main()
