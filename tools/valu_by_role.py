"""Static VALU count of each role of the per-step kernel k_env_step_split<double, false> (flight, ahead, control; the
reset path -- Controller.reset's draws and Model.initialize, one step in 2,000 -- apart) from a gfx950 assembly listing
of the FAST unit built with the product's flags (build.py) and line tables.  An instruction belongs to the role whose
part of the kernel body (b747_split.h: `if (role == 0)`, `if (role == 1)`, the control wave after them) the listing
last referenced, helpers inlined there included; the philox / Box-Muller / initialize lines are the reset path.
Usage: python tools/valu_by_role.py [out.json]   (writes profiles/r06/valu_by_role.json by default)"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "b747_rl_ctrl_amd"))
KERNEL = "_ZN12_GLOBAL__N_116k_env_step_splitIdLb0EE"


def listing(d):
    import build
    flags = [f for f in build.FLAGS if f not in ("-shared", "-fPIC")]
    out = os.path.join(d, "fast.s")
    subprocess.run([build.HIPCC] + flags + ["-gline-tables-only", "--cuda-device-only", "-S", "-o", out,
                                            os.path.join(ROOT, "b747_rl_ctrl_amd", "csrc", "b747_fast.hip")],
                   check=True, capture_output=True)
    return open(out).read().split("\n")


def count(lines):
    files = {}
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln)
        if m:
            files[int(m.group(1))] = os.path.basename(m.group(2))
    st = next(i for i, l in enumerate(lines) if l.startswith(KERNEL))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    src = open(os.path.join(ROOT, "b747_rl_ctrl_amd", "csrc", "b747_split.h")).read().split("\n")

    def find(pat, start=0):
        return next(i + 1 for i in range(start, len(src)) if pat in src[i])
    k0 = find("void k_env_step_split(")
    f0, a0 = find("if (role == 0) {", k0), find("if (role == 1) {", k0)
    c0 = find("// ---- control wave", a0)
    r0 = find("if (valid && rs) {", c0)
    r1 = find("} else if (valid) {", r0)
    role, loc = "prologue", None
    valu, cnd, f64 = collections.Counter(), collections.Counter(), collections.Counter()
    for ln in lines[st:en]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            if loc[0] == "b747_split.h" and loc[1] >= k0:
                role = ("flight" if f0 <= loc[1] < a0 else "ahead" if a0 <= loc[1] < c0 else
                        ("reset" if r0 <= loc[1] < r1 else "control") if loc[1] >= c0 else "prologue")
            continue
        t = ln.strip()
        if not t.startswith("v_"):
            continue
        r = role
        if loc and (loc[0].startswith("__clang") or (loc[0] == "b747_env.h" and loc[1] < 140)):
            r = "reset"
        valu[r] += 1
        cnd[r] += t.startswith("v_cndmask")
        f64[r] += bool(re.match(r"v_(fma|mul|add|rsq|rcp|div_\w+|ldexp|fract)_f64", t))
    return {"valu": dict(valu), "v_cndmask": dict(cnd), "fp64_arith": dict(f64)}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "valu_by_role.json")
    with tempfile.TemporaryDirectory() as d:
        res = count(listing(d))
    res["note"] = ("static instruction counts of k_env_step_split<double, false> per role (tools/valu_by_role.py); "
                   "'reset' is the once-per-episode reset path, 'prologue' the code before the role split")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
