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
                                                os.path.join(ROOT, "include", "b747_tables.h")]
OUT = os.path.join(HERE, "libb747.so")

# -ffp-contract=off: keep the reference DLL's mul/add rounding (no FMA contraction); the FAST
# variant's translation unit (csrc/b747_fast.hip) turns contraction back on with a pragma.
# -disable-machine-licm: stop MachineLICM hoisting ~100 fp64 constants out of the RK4 stage
# loop (it pushed the kernel past 256 VGPRs into AGPR/scratch spills).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-mllvm", "-disable-machine-licm", "-Wall", "-Wno-unused-function"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + SOURCES
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
