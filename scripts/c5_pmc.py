#!/usr/bin/env python3
"""Fold the config-5 PMC passes (scripts/session.sh `pmcs` step: rocprofv3 --pmc of scripts/c5bench.py)
into profiles/c5_pmc.json: per tgms_refine_loop_device call of bench.py's config-5
share, the executed FP64 flops (64 lanes x (ADD + MUL + 2 FMA)), VALU instructions and
HBM bytes (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, MI355X_MICROARCH.md), summed over
the two occupancy-class kernels that one call launches.
    python3 scripts/c5_pmc.py gpurun_out/r05k/pmc_c5bench_default [profiles/c5_pmc.json]"""
import collections, csv, glob, json, re, sys

src = sys.argv[1]
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/c5_pmc.json"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{src}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"(k_refine_loop_(?:multi|dev))<(\d+), (\d+)", k)
        if not m:
            continue
        cls = f"{m.group(1)}<{m.group(2)},{m.group(3)}>"
        acc[cls][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {c: {n: sum(v) / len(v) for n, v in d.items()} for c, d in acc.items()}
tot = collections.Counter()
for d in kern.values():
    tot.update(d)
flops = 64 * (tot["SQ_INSTS_VALU_ADD_F64"] + tot["SQ_INSTS_VALU_MUL_F64"] + 2 * tot["SQ_INSTS_VALU_FMA_F64"])
out = {"c5_share": {"fp64_flops_per_call": flops, "valu_insts_per_call": tot["SQ_INSTS_VALU"],
                    "fp64_insts_per_call": tot["SQ_INSTS_VALU_ADD_F64"] + tot["SQ_INSTS_VALU_MUL_F64"]
                    + tot["SQ_INSTS_VALU_FMA_F64"] + tot["SQ_INSTS_VALU_TRANS_F64"],
                    "hbm_bytes_per_call": tot["FETCH_SIZE"] * 1024 * 2 + tot["WRITE_SIZE"] * 1024,
                    "kernels": kern,
                    "source": f"rocprofv3 --pmc passes of scripts/c5bench.py ({src}), mean per dispatch"}}
try:
    old = json.load(open(dst))
except (OSError, ValueError):
    old = {}
old.update(out)
json.dump(old, open(dst, "w"), indent=1)
print(json.dumps(out["c5_share"], indent=1)[:1500])
