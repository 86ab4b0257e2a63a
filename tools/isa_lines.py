"""Attribute the instructions of one kernel in a `hipcc -S -gline-tables-only` listing to source
lines: python tools/isa_lines.py env.s <kernel-substring> [--loop-depth D] [--top N].
Counts VALU / SALU / LDS / VMEM instructions per (file, line); with --loop-depth only the
instructions of basic blocks at that loop depth (the RK4 stage loop is depth 3 in k_env_steps)."""
import argparse
import collections
import re

ap = argparse.ArgumentParser()
ap.add_argument("asm")
ap.add_argument("kernel")
ap.add_argument("--loop-depth", type=int, default=None)
ap.add_argument("--top", type=int, default=60)
a = ap.parse_args()

files, lines = {}, open(a.asm).read().split("\n")
for ln in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln)
    if m:
        files[int(m.group(1))] = m.group(2).split("/")[-1]
start = next(i for i, ln in enumerate(lines) if re.match(r"^\S*" + re.escape(a.kernel) + r"\S*:", ln))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
loc, depth = ("?", 0), 0
cnt = collections.defaultdict(collections.Counter)
tot = collections.Counter()
body = lines[start:end]
for n, ln in enumerate(body):
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
    if m:
        loc = (files.get(int(m.group(1)), m.group(1)), int(m.group(2)))
        continue
    if re.match(r"^(\.LBB|; %bb)", ln):
        # a loop header's label is followed by "; Parent Loop ... Depth=k" lines: take the deepest
        ds, j = [int(d) for d in re.findall(r"Depth=(\d+)", ln)], n + 1
        while j < len(body) and re.match(r"^\s+;", body[j]):
            ds += [int(d) for d in re.findall(r"Depth=(\d+)", body[j])]
            j += 1
        depth = max(ds) if ds else 0
        continue
    s = ln.strip()
    if not s or s.startswith((";", ".")):
        continue
    op = s.split()[0]
    if a.loop_depth is not None and depth != a.loop_depth:
        continue
    kind = ("LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_"))
            else "SALU" if op.startswith("s_") else "VALU" if op.startswith("v_") else "other")
    cnt[loc][kind] += 1
    cnt[loc]["ops:" + op] += 1
    tot[kind] += 1
print("total", dict(tot))
rows = sorted(cnt.items(), key=lambda kv: -kv[1]["VALU"])
for (f, l), c in rows[: a.top]:
    ops = ",".join(f"{k[4:]}x{v}" for k, v in c.most_common() if k.startswith("ops:v_"))[:110]
    print(f"{f}:{l:<5} VALU {c['VALU']:4d} SALU {c['SALU']:3d} LDS {c['LDS']:2d}  {ops}")
