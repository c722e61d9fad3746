"""CPU: the shipped gfx950 code objects contain no instance of the instruction pair behind
the band-KKT kernel's round-5 wrong-result builds:

    v_cndmask_b32_e64 vX, vConst, vX, s[m:m+1]   ; the lane-selected slab-store offset
    ... fewer than 16 wait states ...
    buffer_store_dwordx2 vData, vX, s[rsrc], s_off offen

Every failing build of round 5 (profiles/r05_band_lane_variants.jsonl: L 128-144 wrong per
run, J 160-267) had it 3-4 states apart; the shipped build separates the two by 16 (two
`s_nop 7` between sched_barriers, tgms_band.hip) and was exact in every run and shape.
The scan (scripts/store_hazard_scan.py) reads the disassembly of each object the build made;
the negative control compiles the band kernel with -DTGMS_BAND_NOGUARD (the unguarded form,
M = 10 only) and finds the pair, so a pass is not an artefact of the scanner."""
import os
import shutil
import subprocess
import sys

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import store_hazard_scan as H  # noqa: E402

MIN_STATES = 16


def _disasm(tmp_path, obj, name):
    fat, co, s = tmp_path / (name + ".fat"), tmp_path / (name + ".co"), tmp_path / (name + ".s")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=%s" % fat, obj],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=%s" % fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=%s" % co], check=True, capture_output=True)
    with open(s, "w") as f:
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)], check=True,
                       stdout=f)
    return str(s)


def _offending(path, kernel=None):
    """(kernel, store, states, producer) for every buffer store whose voffset a v_cndmask wrote
    fewer than MIN_STATES wait states earlier."""
    bad = []
    for name, kern in H.parse(path, kernel).items():
        for r in H.scan(kern, window=MIN_STATES + 8):
            by = r.get("back_addr_by", "")
            if r["op"].startswith("buffer_store") and r["back_addr"] is not None and r["back_addr"] < MIN_STATES \
                    and by.startswith("v_cndmask"):
                bad.append((name, r["op"], r["back_addr"], by))
    return bad


def _need_tools(obj):
    if not os.path.exists(obj) or not shutil.which(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("built objects or LLVM tools absent")


@pytest.mark.parametrize("src", ["tgms_band", "tgms_reduced", "tgms_sample", "tgms_dense"])
def test_shipped_objects_have_no_fresh_select_offset_store(tmp_path, src):
    from trajectory_generator_ros2_amd.build import OBJDIR
    obj = os.path.join(OBJDIR, src + ".hip.o")
    _need_tools(obj)
    s = _disasm(tmp_path, obj, src)
    assert H.parse(s), "no kernels disassembled"
    bad = _offending(s)
    assert not bad, bad[:5]


def test_band_slab_stores_are_16_states_after_any_offset_write(tmp_path):
    """Stronger for the band kernels: EVERY slab buffer store of all 32 instantiations sits at
    least 16 wait states after the last VALU write of its voffset, whatever wrote it."""
    from trajectory_generator_ros2_amd.build import OBJDIR
    obj = os.path.join(OBJDIR, "tgms_band.hip.o")
    _need_tools(obj)
    kerns = H.parse(_disasm(tmp_path, obj, "band"), "k_band_kkt")
    assert len(kerns) == 32
    for name, kern in kerns.items():
        for r in H.scan(kern, window=MIN_STATES + 8):
            if r["op"].startswith("buffer_store"):
                assert r["back_addr"] is None or r["back_addr"] >= MIN_STATES, (name, r)


def test_scanner_finds_the_pair_in_the_unguarded_build(tmp_path):
    """Negative control: the band kernel compiled without the guard (M = 10 only) has the pair."""
    from trajectory_generator_ros2_amd import build as B
    if not shutil.which(B.HIPCC) or not shutil.which(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("hipcc / LLVM tools absent")
    obj = tmp_path / "band_noguard.o"
    subprocess.run([B.HIPCC] + B.HIP_FLAGS + ["-DTGMS_BAND_NOGUARD", "-DTGMS_BAND_ONLY_M10", "-c",
                                              os.path.join(B.CSRC, "tgms_band.hip"), "-o", str(obj)],
                   check=True, capture_output=True)
    bad = _offending(_disasm(tmp_path, str(obj), "band_noguard"), "k_band_kkt")
    assert bad and min(b[2] for b in bad) <= 4, bad[:5]
