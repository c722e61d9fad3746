#!/usr/bin/env python3
"""Scan gfx950 disassembly for the wait-state distance between every vector-memory store
and the VALU instructions around it that write its operands (band-KKT store-offset
failure).  Usage:
    python3 scripts/store_hazard_scan.py FILE.s [KERNEL_SUBSTRING]
FILE.s is `llvm-objdump -d --no-show-raw-insn` output of a gfx950 code object.

For each store it reports
  back_addr   wait states since the last VALU write of its address VGPRs (voffset / vaddr),
  back_data   ... of its data VGPRs,
  back_sgpr   ... since the last VALU write (v_readfirstlane, v_cmp, ...) of its SGPR operands,
  fwd_data    wait states until the next VALU write of its data VGPRs (the store still
              reading them: the ">64-bit store data" hazard),
counting one state per instruction and N+1 for s_nop N, across straight-line code only
(a label or branch ends the window)."""
import re
import sys
from collections import Counter

REG = re.compile(r"\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(a, b + 1))
    return out


def parse(path, kernel=None):
    kerns, cur, name = {}, None, None
    for line in open(path):
        line = line.rstrip()
        if line.endswith(">:"):
            name = line.split("<", 1)[1][:-2]
            cur = kerns.setdefault(name, []) if (kernel is None or kernel in name) else None
            continue
        if cur is None or not line.strip() or line.lstrip().startswith(";"):
            continue
        ins = line.split("//")[0].strip()
        if ins:
            cur.append(ins)
    return kerns


def states(ins):
    if ins.startswith("s_nop"):
        return int(ins.split()[1], 0) + 1
    return 1


def dst_src(ins):
    op, _, rest = ins.partition(" ")
    parts = [p.strip() for p in rest.split(",")]
    if not parts or not parts[0]:
        return op, set(), set()
    if op.startswith(("buffer_store", "global_store", "flat_store", "scratch_store", "ds_write", "s_", "buffer_load_lds",
                      "global_load_lds")):
        return op, set(), regs(rest)
    return op, regs(parts[0]), regs(",".join(parts[1:]))


def is_valu(op):
    return op.startswith("v_")


def scan(kern, window=24):
    rows = []
    for i, ins in enumerate(kern):
        op, _, _ = dst_src(ins)
        if "_store" not in op or op.startswith("ds_") or op.startswith("s_"):
            continue
        _, rest = ins.split(" ", 1)
        ops = [p.strip() for p in rest.split(",")]
        if op.startswith("buffer_store"):
            data, addr, sg = regs(ops[0]), regs(ops[1]), regs(ops[2]) | regs(ops[3].split()[0])
        else:  # global_store vaddr, data, saddr/off
            addr, data = regs(ops[0]), regs(ops[1])
            sg = regs(ops[2].split()[0]) if len(ops) > 2 else set()
        res = {"i": i, "op": op}
        for key, want in (("back_addr", addr), ("back_data", data), ("back_sgpr", sg)):
            d, j = 0, i - 1
            res[key] = None
            while j >= 0 and d < window:
                o2, dst, _ = dst_src(kern[j])
                if o2.startswith("s_cbranch") or o2.startswith("s_branch"):
                    break
                if is_valu(o2) and dst & want:
                    res[key] = d
                    res[key + "_by"] = kern[j]
                    break
                d += states(kern[j])
                j -= 1
        d, j = 0, i + 1
        res["fwd_data"] = None
        while j < len(kern) and d < window:
            o2, dst, _ = dst_src(kern[j])
            if o2.startswith("s_cbranch") or o2.startswith("s_branch"):
                break
            if is_valu(o2) and dst & data:
                res["fwd_data"] = d
                res["fwd_data_by"] = kern[j]
                break
            d += states(kern[j])
            j += 1
        rows.append(res)
    return rows


def main():
    path = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else None
    for name, kern in parse(path, kernel).items():
        rows = scan(kern)
        if not rows:
            continue
        print(name, "stores:", len(rows))
        for key in ("back_addr", "back_data", "back_sgpr", "fwd_data"):
            c = Counter(r[key] for r in rows if r[key] is not None)
            print("  %-9s min %s  hist %s" % (key, min(c) if c else None, sorted(c.items())[:8]))
        for r in rows:
            close = [k for k in ("back_addr", "back_sgpr", "fwd_data") if r[k] is not None and r[k] < 3]
            if close:
                print("   ", r["op"], {k: (r[k], r.get(k + "_by")) for k in close})


if __name__ == "__main__":
    main()
