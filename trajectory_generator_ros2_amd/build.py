"""In-tree build of libtgms.so (HIP, gfx950) and of the C++ host adapter.

The shared libraries are written next to the sources (``lib/``) so they travel to
the GPU box with the repository snapshot.  Nothing here touches the oracle.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
HOST = os.path.join(PKG, "host")
LIBDIR = os.path.join(PKG, "lib")
INCLUDE = os.path.join(ROOT, "include")
OBJDIR = os.path.join(PKG, "build")

LIB_TGMS = os.path.join(LIBDIR, "libtgms.so")
LIB_HOST = os.path.join(LIBDIR, "libtgms_node.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TGMS_ARCH", "gfx950")
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-I" + CSRC]

HIP_SOURCES = ["tgms_reduced.hip", "tgms_dense.hip", "tgms_band.hip", "tgms_sample.hip", "tgms_capi.hip"]
CXX_SOURCES = ["tgms_plan.cpp", "tgms_host.cpp"]  # host-only (no HIP): compiled by g++ into the same library
HOST_SOURCES = ["MinSnap.cpp", "factory.cpp", "tgms_node_capi.cpp"]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r


def _headers():
    hs = [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    hs += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs


def build_tgms(force: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    objs = [os.path.join(OBJDIR, os.path.basename(s) + ".o") for s in srcs]
    hdrs = _headers()
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _newer(o, [s] + hdrs)]
    csrcs = [os.path.join(CSRC, s) for s in CXX_SOURCES]
    cobjs = [os.path.join(OBJDIR, os.path.basename(s) + ".o") for s in csrcs]
    ctodo = [(s, o) for s, o in zip(csrcs, cobjs) if force or _newer(o, [s] + hdrs)]
    cxx = ["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-I" + INCLUDE, "-I" + CSRC]
    with ThreadPoolExecutor(max_workers=len(srcs) + len(csrcs)) as ex:
        jobs = [ex.submit(_run, [HIPCC] + HIP_FLAGS + ["-c", s, "-o", o]) for s, o in todo]
        jobs += [ex.submit(_run, cxx + ["-c", s, "-o", o]) for s, o in ctodo]
        for j in jobs:
            j.result()
    objs = objs + cobjs
    todo = todo + ctodo
    if force or todo or _newer(LIB_TGMS, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB_TGMS] + objs + ["-ldl"])
    return LIB_TGMS


def build_host(force: bool = False) -> str:
    """C++ MinSnap adapter (mirror of the reference Trajectory interface) -> libtgms_node.so."""
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = [os.path.join(HOST, s) for s in HOST_SOURCES]
    if not all(os.path.exists(s) for s in srcs):
        return ""
    hdrs = [os.path.join(HOST, f) for f in os.listdir(HOST) if f.endswith((".hpp", ".h"))] + _headers()
    if force or _newer(LIB_HOST, srcs + hdrs + [LIB_TGMS]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-I" + INCLUDE, "-I" + HOST,
              "-o", LIB_HOST] + srcs + ["-L" + LIBDIR, "-ltgms", "-Wl,-rpath,$ORIGIN"])
    return LIB_HOST


def build(force: bool = False) -> None:
    build_tgms(force)
    build_host(force)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB_TGMS)
