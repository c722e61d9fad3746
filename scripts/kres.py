#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
    python3 scripts/kres.py <file.hip> [filter] [-D...]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
       "-Itrajectory_generator_ros2_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + defs
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = re.sub(r"_ZN4tgms12_GLOBAL__N_1\d+", "", v)[:60]
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt in name:
        print(f"{name:60s} vgpr {r.get('VGPRs','?'):>4} spill {r.get('VGPRs Spill','?'):>3} "
              f"sgpr-spill {r.get('SGPRs Spill','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?'):>2} "
              f"lds {r.get('LDS Size [bytes/block]','?')}")
