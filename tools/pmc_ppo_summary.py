"""Per-wave SQ counters of the fused config-5 rollout kernel from a tools/pmc_ppo.sh profile.

Usage: python tools/pmc_ppo_summary.py gpurun_out/ppo_sq/prof profiles/r02
Writes <out>/ppo_rollout_sq_counters.json: counters summed over each k_ppo_rollout dispatch, divided
by its SQ_WAVES, averaged over the dispatches after the first (a dispatch = one 64-step rollout, so
the per-wave figures cover 64 env steps; `per_wave_per_step` divides them by the rollout length).
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("k_ppo_rollout", "k_rollout_split<true")   # the one-wave and the two-wave (policy) rollout kernels
STEPS = 64

src, out = sys.argv[1], sys.argv[2]
path = next(p for p in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True))
agg = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    if not any(k in r["Kernel_Name"] for k in KERNELS):
        continue
    d = agg.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
    d[r["Counter_Name"]] += float(r["Counter_Value"])
rows = list(agg.values())[1:]
names = sorted(k for k in rows[0] if k != "SQ_WAVES")
per_wave = {k: statistics.mean(d[k] / d["SQ_WAVES"] for d in rows) for k in names}
res = {
    "kernel": "k_rollout_split<true, double> (b747_ppo_rollout)",
    "dispatches": len(rows),
    "waves": statistics.mean(d["SQ_WAVES"] for d in rows),
    "rollout_steps": STEPS,
    "per_wave": per_wave,
    "per_wave_per_step": {k: v / STEPS for k, v in per_wave.items()},
    "valu_issue_frac": per_wave["SQ_ACTIVE_INST_VALU"] / per_wave["SQ_WAVE_CYCLES"],
    "wait_any_frac": per_wave["SQ_WAIT_ANY"] / per_wave["SQ_WAVE_CYCLES"],
    "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are in quad-cycles (x4 = clock cycles)",
}
os.makedirs(out, exist_ok=True)
with open(os.path.join(out, "ppo_rollout_sq_counters.json"), "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
