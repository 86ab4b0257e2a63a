"""Per-kernel resources of a built library's gfx950 code object (AMDGPU metadata notes): VGPRs, AGPRs, spills,
scratch bytes per lane, LDS bytes.  Usage: python tools/kernel_resources.py [lib.so] [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(so, d):
    fb = os.path.join(d, "fb.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", so, os.path.join(d, "copy.so")],
                   check=True)   # (an explicit output: without one llvm-objcopy rewrites the library in place)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    for k, s0 in enumerate(starts):
        part, co = os.path.join(d, f"b{k}.bin"), os.path.join(d, f"co{k}.o")
        open(part, "wb").write(data[s0:starts[k + 1] if k + 1 < len(starts) else len(data)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"], check=True)
        yield co


def resources(so):
    """{demangled kernel name: {field: value}} from the code objects' metadata notes"""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(so, d):
            txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                 text=True).stdout
            for blk in re.split(r"\n  - (?=\.agpr_count:)", txt):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or ".vgpr_count" not in blk:
                    continue
                f = {}
                for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                            "private_segment_fixed_size", "group_segment_fixed_size"):
                    mm = re.search(r"\." + key + r":\s+(\d+)", blk)
                    f[key] = int(mm.group(1)) if mm else None
                out[m.group(1)] = f
    names = list(out)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return {dn: out[n] for n, dn in zip(names, dem)}


def main(argv):
    so = argv[0] if argv and argv[0].endswith(".so") else os.path.join(ROOT, "b747_rl_ctrl_amd", "libb747.so")
    pats = [a for a in argv if not a.endswith(".so")]
    res = resources(so)
    for name, f in sorted(res.items()):
        if pats and not any(p in name for p in pats):
            continue
        short = re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]
        print(f"{short[:60]:60s} vgpr {f['vgpr_count']:3d} agpr {f['agpr_count']:3d} spill v{f['vgpr_spill_count']} "
              f"s{f['sgpr_spill_count']} scratch {f['private_segment_fixed_size']:4d} lds {f['group_segment_fixed_size']}")
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
