"""Build properties the measured kernel times depend on, checked on the CPU from the shipped gfx950 code object
(DESIGN.md 4): a change that silently breaks one of them keeps every parity test green and only shows up as a
slower bench line on the GPU.
  * the per-step kernel (k_env_step_split, 256 envs per workgroup) runs three waves per SIMD: at most 168 VGPRs
    (512 / 3 rounded down to the allocation granule of 8), no scratch (its small-batch form, 64 envs: no scratch);
  * its leading arguments (n and six state pointers) arrive preloaded in SGPRs (-amdgpu-kernarg-preload-count=14,
    build.py): the code object then starts with the firmware-compatibility prologue that loads them itself and
    branches over the 256-byte pad to the kernel proper;
  * the K-step rollout kernels (k_rollout_split<false, ...>, 256 envs per workgroup) fit two waves per SIMD without
    scratch (the 64-env small-batch forms: no scratch)."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "b747_rl_ctrl_amd", "libb747.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"),
                                reason="needs the built library and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def res():
    import kernel_resources
    return kernel_resources.resources(LIB)


def _pick(res, pat):
    got = {n: f for n, f in res.items() if pat in n}
    assert got, f"no kernel matching {pat!r} in {LIB}"
    return got


def test_per_step_kernel_fits_three_waves_per_simd(res):
    got = _pick(res, "k_env_step_split<")
    assert len(got) == 8, sorted(got)   # fp64 / fp32 storage x FAST / MIXED x 256 / 64 envs per workgroup
    for name, f in got.items():
        # 256 envs per workgroup (the bench's 65,536 envs): three waves per SIMD; the small-batch form (64 envs, one
        # wave of each role per SIMD) may use up to a full SIMD's registers
        if ", 256>" in name:
            assert f["vgpr_count"] + (f["agpr_count"] or 0) <= 168, (name, f)
        assert f["private_segment_fixed_size"] == 0 and f["vgpr_spill_count"] == 0, (name, f)


def test_k_step_rollout_fits_two_waves_per_simd(res):
    for name, f in _pick(res, "k_rollout_split<false").items():
        if ", 256>" in name:   # (the small-batch form, 64 envs per workgroup, runs one wave per SIMD)
            assert f["vgpr_count"] + (f["agpr_count"] or 0) <= 256, (name, f)
        assert f["private_segment_fixed_size"] == 0, (name, f)


def test_per_step_kernel_arguments_are_preloaded():
    import isa_pk_hazard as H
    seen = 0
    for name, body in H.kernels(LIB):
        if "k_env_step_split" not in name:
            continue
        seen += 1
        # the compatibility prologue: the preloaded argument SGPRs loaded from the segment, then a jump over the pad
        head = body[:6]
        loads = [s for s in head if s.startswith("s_load_")]
        assert loads and re.match(r"s_load_dwordx2 s\[2:3\], s\[0:1\], 0x0", loads[0]), (
            f"{name}: no kernel-argument preload prologue -- did this ROCm drop -mllvm -amdgpu-kernarg-preload-count=14 "
            f"(build.py, INTEGRATION.md §8)?", head)
        assert any(s.startswith("s_branch") for s in head), (name, head)
        width = sum(int(re.match(r"s_load_dword(?:x(\d+))?", s).group(1) or 1) for s in loads)
        assert width == 14, (name, head)   # n (2 dwords) + six 64-bit pointers
    assert seen == 8   # double / float storage x FAST / MIXED x 256 / 64 envs per workgroup


def test_model_split_kernels_have_no_scratch(res):
    """The model API's three-wave kernels (b747_model_split.h; one wave per role per SIMD at config 2's size): no
    scratch (a refactor of their signal writes once cost the K-step fp64 instantiation 68 B of it)."""
    for pat in ("k_model_step_split<", "k_model_steps_split<"):
        for name, f in _pick(res, pat).items():
            assert f["private_segment_fixed_size"] == 0 and f["vgpr_spill_count"] == 0, (name, f)
