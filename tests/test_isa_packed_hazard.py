"""The shipped gfx950 code has no packed-fp32 read-after-write of the kind that broke the packed layer 1.

VERDICT r2 #5, root cause (tools/exp_l1_packed.py on MI355X): the round-2 experiment's VALU
layer 1 with two hidden units per v_pk_fma_f32 gave wrong results in lanes 48-63 of EVERY wave (a quarter
of all envs, both heads; the earlier "one wave of four" was that quarter).  The same packed FMAs written
as inline asm, each followed by an s_nop so that its result is read 2 or more wait states later, are
correct in every lane; the compiler's own schedule reads v_pk_fma_f32 results after 1 wait state (by
v_pk_fma_f32, v_fma_f32 and v_exp_f32).  The shipped kernels have no v_pk_fma_f32 / v_pk_mul_f32; the only
packed-fp32 results they read that early are v_pk_add_f32's (the f16 hi/lo split: lo = x - hi) read by
v_cvt_pk_f16_f32, a pair the GPU parity tests check in every lane (tests/test_gpu_ppo.py,
tests/test_gpu_fullsize.py).  This test keeps it that way: any other early read of a packed-fp32 result
in libb747.so fails here, on the CPU, before it can fail a quarter of the lanes on the GPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "b747_rl_ctrl_amd", "libb747.so")

VERIFIED = {("v_pk_add_f32", "v_cvt_pk_f16_f32")}   # (writer, reader) checked in every lane on the GPU


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_unverified_early_read_of_a_packed_fp32_result():
    import isa_pk_hazard as H
    bad = H.main([LIB])
    seen = set()
    for name, hits in bad.items():
        for (ws, reader, writer), n in hits.items():
            seen.add((writer, reader))
            assert (writer, reader) in VERIFIED, (f"{name}: {writer} result read by {reader} after {ws} wait "
                                                  f"state(s) ({n}x): the packed-fp32 hazard of DESIGN.md 4")
    assert "v_pk_fma_f32" not in {w for w, _ in seen}
