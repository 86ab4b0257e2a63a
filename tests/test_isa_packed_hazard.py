"""The shipped gfx950 code reads no packed-fp32 or transcendental result early.

Root cause (profiles/r03/packed_layer1_root_cause.txt on MI355X): the round-2 experiment's VALU layer 1 with two hidden
units per v_pk_fma_f32 gave wrong results in lanes 48-63 of EVERY wave; the same packed FMAs as inline asm, each
followed by an s_nop so that its result is read 2 or more wait states later, are correct in every lane, and
packed head sums as inline asm that read v_rcp_f32 results the compiler did not see being read were wrong in the
same lanes.  This compiler (ROCm 7.2 LLVM) pads a transcendental result's first use to 1 wait state in code it
schedules itself (hundreds of such reads in the shipped tanh and division code pass every lane of the GPU parity
tests), but gives a packed-fp32 result only the same 1 where 2 are needed.
Round 4 removed the last early packed read of the shipped kernels -- the f16 hi/lo split's lo = x - hi
(v_pk_add_f32 read by v_cvt_pk_f16_f32 one wait state later, until then "verified" by the GPU parity tests) --
by construction: split_pair's packed subtraction is inline asm followed by s_nop 1, and the observation split's
subtraction a scalar v_sub_f32 (csrc/b747_policy.h).  So the list of tolerated patterns is empty: any early read
of a packed-fp32 or transcendental result in libb747.so fails here, on the CPU, before it can fail a quarter of
the lanes on the GPU, and so does any transcendental result read with no wait state at all."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "b747_rl_ctrl_amd", "libb747.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_early_read_of_a_packed_fp32_or_transcendental_result():
    import isa_pk_hazard as H
    assert "v_rcp_f32" in H.WRITERS and "v_pk_add_f32" in H.WRITERS and H.MIN_WS == 2 and H.MIN_WS_TRANS == 1
    bad = H.main([LIB])
    found = [f"{name[:80]}: {writer} read by {reader} after {ws} wait state(s) x{n}"
             for name, hits in bad.items() for (ws, reader, writer), n in hits.items()]
    assert not found, "the gfx950 early-read hazard of DESIGN.md 4:\n" + "\n".join(found)


def test_the_scan_finds_the_pattern():
    """The scanner itself: a packed write read one instruction later is early, s_nop 1 in between is not; a
    transcendental result read by the next instruction is early, one instruction later is not."""
    import isa_pk_hazard as H

    def early(body):
        return {k: v for k, v in H.scan(body).items() if k[0] < H.min_ws(k[2])}
    assert early(["v_pk_add_f32 v[4:5], v[0:1], v[2:3]", "v_cvt_pk_f16_f32 v6, v4, v5"])
    assert early(["v_pk_add_f32 v[4:5], v[0:1], v[2:3]", "s_nop 0", "v_cvt_pk_f16_f32 v6, v4, v5"])
    assert not early(["v_pk_add_f32 v[4:5], v[0:1], v[2:3]", "s_nop 1", "v_cvt_pk_f16_f32 v6, v4, v5"])
    assert early(["v_rcp_f32_e32 v3, v2", "v_fma_f32 v4, v3, v1, v0"])      # (objdump's encoding suffixes)
    assert not early(["v_exp_f32_e32 v3, v2", "v_mov_b32_e32 v9, v8", "v_fma_f32 v4, v3, v1, v0"])
