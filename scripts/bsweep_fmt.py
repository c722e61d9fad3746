#!/usr/bin/env python3
"""One line per kbench.py JSON record on stdin."""
import json, sys
for l in sys.stdin:
    l = l.strip()
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    if "lib" not in d:
        print(l); continue
    print(f"{d['lib']:24s} B={d['B']:7d} rot={d.get('rot', 1)} med {d['median_us']:8.1f} min {d['min_us']:8.1f} "
          f"err {d['max_rel_err']:.1e}")
