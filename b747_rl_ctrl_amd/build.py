"""Build libb747.so (HIP, gfx950) in-tree with hipcc.  Used by __graft_entry__.build()."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("B747_OFFLOAD_ARCH", "gfx950")

SOURCES = [os.path.join(HERE, "csrc", "b747_kernels.hip"), os.path.join(HERE, "csrc", "b747_fast.hip")]
DEPS = SOURCES + sorted(os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))
                        if f.endswith(".h")) + [os.path.join(ROOT, "include", "b747.h"),
                                                os.path.join(ROOT, "include", "b747_tables.h"),
                                                os.path.join(ROOT, "include", "b747_isa_cells.h")]
OUT = os.path.join(HERE, "libb747.so")
# the reference DLL's exported-globals ABI over libb747.so (core/model.py loads `model_simple.so` on Linux)
SHIM_SRC = os.path.join(HERE, "csrc", "model_simple_gpu.cpp")
SHIM = os.path.join(HERE, "model_simple.so")

# -ffp-contract=off: keep the reference DLL's mul/add rounding (no FMA contraction); the FAST
# variant's translation unit (csrc/b747_fast.hip) turns contraction back on with a pragma.
# -disable-machine-licm: stop MachineLICM hoisting ~100 fp64 constants out of the RK4 stage
# loop (it pushed the kernel past 256 VGPRs into AGPR/scratch spills).
# -amdgpu-kernarg-preload-count=14: the dispatch places a kernel's leading scalar/pointer arguments (14 dwords) in
# SGPRs; the per-step kernel leads with the pointers its first loads need (b747_split.h: 9.11-9.26 against
# 9.26-9.38 us per step, A/B on one box).  Kernels that lead with a struct argument preload nothing.
# -fno-slp-vectorize: no compiler-made packed fp32 (v_pk_mul/add/fma_f32): this compiler reads their results one wait
# state after the write, where gfx950 needs two (lanes 48-63 see stale values; DESIGN.md 4,
# tests/test_isa_packed_hazard.py) -- the MIX flight pass's fp32 arithmetic would otherwise be paired up.
# -amdgpu-sched-strategy=max-ilp: the machine scheduler's latency-first strategy; the per-step kernel 8.54-8.56 against
# 8.63-8.68 us in rocprofv3 (3 interleaved rounds, one box; the rollout kernels within noise: profiles/r06/ab_step_kernel.txt).
# All three -mllvm flags are LLVM-internal options, not a stable interface.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-mllvm", "-disable-machine-licm", "-fno-slp-vectorize",
         "-mllvm", "-amdgpu-kernarg-preload-count=14",
         "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-Wall", "-Wno-unused-function"]


def _src_hash(deps, flags):
    """sha256 over the sources' contents and the compile command: the build is redone whenever they change (file
    mtimes are not trusted -- copies, checkouts and snapshots move them either way)"""
    import hashlib
    h = hashlib.sha256(" ".join(flags).encode())
    for d in deps:
        h.update(d.encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _file_hash(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def needs_build(out=OUT, deps=DEPS, flags=FLAGS):
    """The stamp holds the sources' hash and the built file's own: a library replaced after the build (a copied
    variant, a partial write) no longer matches and is rebuilt"""
    stamp = out + ".srchash"
    if not os.path.exists(out) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        got = f.read().split()
    return got != [_src_hash(deps, flags), _file_hash(out)]


def _write_stamp(out, deps, flags):
    with open(out + ".srchash", "w") as f:
        f.write(_src_hash(deps, flags) + " " + _file_hash(out) + "\n")


def build_shim(force=False, verbose=True):
    """model_simple.so: host code only (no kernels), linked against libb747.so (rpath: see below)."""
    deps = [SHIM_SRC, OUT, os.path.join(ROOT, "include", "b747.h"), os.path.join(ROOT, "include", "b747_tables.h")]
    if not force and not needs_build(SHIM, deps, []):
        return SHIM
    cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wall", f"-I{os.path.join(ROOT, 'include')}", "-o", SHIM,
           SHIM_SRC, f"-L{HERE}", "-lb747",
           # core/model.py:99-113 loads a COPY of the library from core/tmp_models/<uuid>.so: libb747.so is
           # found beside the original ($ORIGIN/.. from tmp_models), beside the copy, or in this build dir
           "-Wl,-rpath,$ORIGIN/..:$ORIGIN:" + HERE]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    _write_stamp(SHIM, deps, [])
    return SHIM


def build(force=False, verbose=True):
    if force or needs_build():
        cmd = [HIPCC] + FLAGS + ["-o", OUT] + SOURCES
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        _write_stamp(OUT, DEPS, FLAGS)
    build_shim(force, verbose)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
