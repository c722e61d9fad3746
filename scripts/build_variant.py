#!/usr/bin/env python3
"""Kernel experiments: build lib/variants/libtgms_<name>.so = libtgms.so with one HIP source
recompiled under extra defines (e.g. ablations).  Usage:
  python3 scripts/build_variant.py NAME SOURCE.hip[,SOURCE2.hip] -DFLAG [-DFLAG2 ...]"""
import os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trajectory_generator_ros2_amd import build as B

name, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
B.build_tgms()
vdir = os.path.join(B.LIBDIR, "variants")
os.makedirs(vdir, exist_ok=True)
srcs = src.split(",")  # several sources: comma-separated
vobjs = []
for sname in srcs:
    obj = os.path.join(B.OBJDIR, "variant_%s_%s.o" % (name, os.path.basename(sname)))
    B._run([B.HIPCC] + B.HIP_FLAGS + flags + ["-c", os.path.join(B.CSRC, sname), "-o", obj])
    vobjs.append(obj)
bases = [os.path.basename(s) for s in srcs]  # (a source may be an absolute path: a saved older version)
objs = [os.path.join(B.OBJDIR, s + ".o") for s in B.HIP_SOURCES + B.CXX_SOURCES if s not in bases] + vobjs
out = os.path.join(vdir, "libtgms_%s.so" % name)
B._run([B.HIPCC, "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o", out] + objs + ["-ldl"])
print(out)
