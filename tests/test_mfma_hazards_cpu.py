"""The inline-asm weight-gradient MFMAs of csrc/mbwave.hip (mfma4_acc) are invisible to LLVM's
hazard recognizer; tools/mfma_hazards.py audits their wait states on the device listing of every
kernel instantiation (the Makefile runs it before linking libdppo.so).  Here: the audit itself
catches each hazard class on hand-written listings, and the shipped kernels pass it."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import mfma_hazards as MH  # noqa: E402

MFMA = "v_mfma_f32_16x16x4_f32 a[0:3], {a}, {b}, a[0:3]"


def _listing(tmp_path, body):
    lines = ["_Zk:"]
    for ln in body:
        if ln.startswith("asm "):
            lines += ["\t;;#ASMSTART", "\t" + ln[4:], "\t;;#ASMEND"]
        elif ln.startswith("."):
            lines.append(ln)
        else:
            lines.append("\t" + ln)
    lines += ["\ts_endpgm", ".Lfunc_end0:"]
    p = tmp_path / "k.s"
    p.write_text("\n".join(lines) + "\n")
    ks = MH.parse(str(p))
    return sorted({v[0] for v in MH.check("_Zk", ks["_Zk"])})


def test_valu_write_to_asm_mfma_operand(tmp_path):
    assert _listing(tmp_path, ["v_mul_f32_e32 v1, v2, v3", "asm " + MFMA.format(a="v1", b="v4")]) == ["R1"]
    assert _listing(tmp_path, ["v_mul_f32_e32 v1, v2, v3", "s_nop 1",
                               "asm " + MFMA.format(a="v1", b="v4")]) == []


def test_asm_mfma_result_read_too_early(tmp_path):
    body = ["asm " + MFMA.format(a="v5", b="v4"), "s_nop 7", "v_accvgpr_read_b32 v9, a2"]
    assert _listing(tmp_path, body) == ["R2"]
    body = ["asm " + MFMA.format(a="v5", b="v4"), "s_nop 7", "s_nop 3", "v_accvgpr_read_b32 v9, a2"]
    assert _listing(tmp_path, body) == []
    # accumulate chain: the next asm MFMA on the same tuple needs no states
    assert _listing(tmp_path, ["asm " + MFMA.format(a="v5", b="v4"),
                               "asm " + MFMA.format(a="v6", b="v4")]) == []


def test_srcc_overwritten_too_early(tmp_path):
    body = ["asm " + MFMA.format(a="v5", b="v4"), "s_nop 7", "s_nop 7", "v_accvgpr_write_b32 a1, v3"]
    assert _listing(tmp_path, body) == []
    body = ["asm " + MFMA.format(a="v5", b="v4"), "s_nop 3", "v_accvgpr_write_b32 a1, v3"]
    assert set(_listing(tmp_path, body)) == {"R2", "R3"}


def test_hazard_across_loop_back_edge(tmp_path):
    body = [".LBB0_1:   ; =>This Inner Loop Header: Depth=1", "v_accvgpr_read_b32 v9, a2",
            "s_nop 7", "s_nop 7",
            "asm " + MFMA.format(a="v5", b="v4"), "s_cbranch_scc1 .LBB0_1"]
    assert _listing(tmp_path, body) == ["R2"]
    body = [".LBB0_1:", "s_nop 7", "s_nop 3", "v_accvgpr_read_b32 v9, a2",
            "asm " + MFMA.format(a="v5", b="v4"), "s_cbranch_scc1 .LBB0_1"]
    assert _listing(tmp_path, body) == []


CMFMA = "v_mfma_f32_16x16x4_f32 v[10:13], {a}, {b}, v[20:23]"


def test_asm_valu_rules(tmp_path):
    """Inline-asm VALU (the DPPO_MBW_PK_ASM form of the packed steps) against the compiler's own
    MFMAs, transcendentals and lane moves, which the recognizer cannot pair with it."""
    pk = "v_pk_mul_f32 v[2:3], v[4:5], v[6:7]"
    # R4: asm VALU result read by a compiler MFMA
    assert _listing(tmp_path, ["asm " + pk, CMFMA.format(a="v2", b="v8")]) == ["R4"]
    assert _listing(tmp_path, ["asm " + pk, "s_nop 1", CMFMA.format(a="v2", b="v8")]) == []
    # R5: a transcendental result read by asm VALU
    assert _listing(tmp_path, ["v_exp_f32_e32 v4, v9", "asm " + pk]) == ["R5"]
    assert _listing(tmp_path, ["v_exp_f32_e32 v4, v9", "s_nop 1", "asm " + pk]) == []
    # R6: a compiler MFMA result read by asm VALU
    body = [CMFMA.format(a="v30", b="v31"), "s_nop 3", "asm v_pk_mul_f32 v[2:3], v[10:11], v[6:7]"]
    assert _listing(tmp_path, body) == ["R6"]
    body = [CMFMA.format(a="v30", b="v31"), "s_nop 7", "s_nop 3",
            "asm v_pk_mul_f32 v[2:3], v[10:11], v[6:7]"]
    assert _listing(tmp_path, body) == []
    # R7: asm VALU overwriting a compiler MFMA's SrcC while it is read
    body = [CMFMA.format(a="v30", b="v31"), "asm v_pk_mul_f32 v[20:21], v[4:5], v[6:7]"]
    assert _listing(tmp_path, body) == ["R7"]
    # R8: asm VALU result read by a lane move
    assert _listing(tmp_path, ["asm " + pk, "v_permlane16_swap_b32_e32 v2, v3"]) == ["R8"]


def test_shipped_minibatch_kernels_pass_the_audit():
    pkg = os.path.join(ROOT, "diamond-ppo_amd")
    subprocess.run(["make", "-C", pkg, "build/mbwave.s"], check=True, capture_output=True)
    listing = os.path.join(pkg, "build", "mbwave.s")
    ks = MH.parse(listing)
    n_asm = sum(1 for items in ks.values() for it in items
                if it[0] == "ins" and it[2] and it[1].startswith("v_mfma"))
    assert n_asm > 0, "no inline-asm MFMA found: the audit would be vacuous"
    bad = [v for k, items in ks.items() for v in MH.check(k, items)]
    assert not bad, bad[:10]
