"""The DPP instruction forms of the built kernels (tools/isa_dpp.py) are the ones the GPU parity
suite verified, and none is a form MI355X executes differently from the compiler's model.

DPP moves that exchange values between lanes can be folded by the compiler (GCNDPPCombine) into
the VOP2 instruction that consumes them; the DPP lane select then applies to that instruction's
src0.  On MI355X a REVERSED VOP2 opcode with DPP -- v_subrev_u32_dpp, v_lshlrev_b32_dpp -- applies
the lane select to src1 instead: tools/dpp/dpp_fold_test.hip runs each encoded form on the GPU
(encodings checked field by field: the DPP word's src0 is the intended register), and every
*rev* case returns exactly "the same operation with the lane select on src1"
(profiles/r06_e_dpp_fold_test.txt); v_add / v_sub / v_and / v_or / v_mov with DPP are exact.
That is round 5's miscompile: the lane ^ 1 low / high moves (quad_perm [0,0,2,2] / [1,1,3,3])
folded into v_subrev_u32_dpp gave wrong residuals.  This test runs on the
CPU against the library built in the tree: a reversed opcode with DPP fails it outright, and any
other form outside the verified set fails until it is re-verified on MI355X (pytest -m gpu + the
fold micro-test) and added below.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_dpp  # noqa: E402

LIB = os.path.join(ROOT, "arrow-h264_amd", "lib", "libh264r.so")

FULL = "row_mask:0xf bank_mask:0xf"
# (mnemonic, modifiers) the parity suite exercises today
VERIFIED = {
    # lane_xor1, quad_bcast<K> as moves
    ("v_mov_b32_dpp", f"quad_perm:[1,0,3,2] {FULL}"),
    ("v_mov_b32_dpp", f"quad_perm:[0,0,0,0] {FULL}"),
    ("v_mov_b32_dpp", f"quad_perm:[1,1,1,1] {FULL}"),
    ("v_mov_b32_dpp", f"quad_perm:[2,2,2,2] {FULL}"),
    ("v_mov_b32_dpp", f"quad_perm:[3,3,3,3] {FULL}"),
    # lane_lo4 / lane_hi4 (and lane_xor4's two halves): banked row shifts keeping the own value,
    # verified only as separate moves -- a fold of these into a VOP2 is a new form
    ("v_mov_b32_dpp", "row_shl:4 row_mask:0xf bank_mask:0x5"),
    ("v_mov_b32_dpp", "row_shr:4 row_mask:0xf bank_mask:0xa"),
    # folds the suite verifies: lane_xor1 into an AND, quad_bcast<0> into an ADD
    ("v_and_b32_dpp", f"quad_perm:[1,0,3,2] {FULL} bound_ctrl:1"),
    ("v_add_u32_dpp", f"quad_perm:[0,0,0,0] {FULL} bound_ctrl:1"),
    # k_level's wave-wide OR (the compiler's reduction of its ballot / max loop)
    ("v_mov_b32_dpp", f"wave_shl:1 {FULL} bound_ctrl:1"),
    ("v_or_b32_dpp", f"{FULL} bound_ctrl:1"),
    ("v_or_b32_dpp", f"row_shl:1 {FULL} bound_ctrl:1"),
    ("v_or_b32_dpp", f"row_shl:2 {FULL} bound_ctrl:1"),
    ("v_or_b32_dpp", f"row_shl:4 {FULL} bound_ctrl:1"),
    ("v_or_b32_dpp", f"row_shl:8 {FULL} bound_ctrl:1"),
}


@pytest.fixture(scope="module")
def forms():
    if not os.path.exists(LIB):
        pytest.skip("libh264r.so not built (__graft_entry__.build())")
    return isa_dpp.dpp_forms(LIB)


def test_every_dpp_form_is_a_verified_one(forms):
    new = sorted({(k, op, mods) for (k, op, mods) in forms if (op, mods) not in VERIFIED})
    assert not new, "DPP forms the GPU parity suite has not verified: " + "; ".join(f"{k}: {op} {m}" for k, op, m in new)


def test_no_lane1_low_high_move_is_folded(forms):
    """The round-5 miscompile's family: quad_perm [0,0,2,2] / [1,1,3,3] in anything but a move."""
    bad = [(k, op, m) for (k, op, m) in forms
           if ("quad_perm:[0,0,2,2]" in m or "quad_perm:[1,1,3,3]" in m) and op != "v_mov_b32_dpp"]
    assert not bad, bad


def test_lane_lo4_hi4_stay_moves(forms):
    """lane_lo4 / lane_hi4 (device_common.h): the banked row shifts (bank_mask 0x5 / 0xa) appear, and
    only as separate v_mov_b32_dpp moves."""
    banked = [(k, op) for (k, op, m) in forms if "bank_mask:0x5" in m or "bank_mask:0xa" in m]
    assert banked
    assert all(op == "v_mov_b32_dpp" for _, op in banked), banked


def test_no_dpp_on_a_reversed_opcode(forms):
    """v_*rev*_dpp (subrev, lshlrev, lshrrev, ashrrev, ...): MI355X applies the lane select to src1."""
    bad = sorted({(k, op, m) for (k, op, m) in forms if "rev_" in op})
    assert not bad, bad
