"""Summarise a rocprofv3 profile of bench.py into profiles/<round>/ (committed evidence).

Reads a directory produced by tools/gpu_round.sh (trace_kernel_stats.csv, pmc_FETCH_SIZE_*,
pmc_WRITE_SIZE_*, pmc_sq_*), and writes
  env_step_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (copied)
  env_step_pmc_traffic.json      per-launch HBM-side bytes of the env-step kernel:
                                 FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md "HBM")
                                 + WRITE_SIZE, averaged over the dispatches after warm-up
  env_step_sq_counters.json      SQ counters per wave (instruction mix, wait cycles)
Usage: python tools/pmc_summary.py gpurun_out/r01e/prof profiles/r01 [--envs 65536]
"""
import argparse
import collections
import csv
import json
import os
import shutil
import statistics

KERNEL = "k_env_step"   # k_env_steps (one wave per env) and k_env_step_split (two)


def per_dispatch(path, skip=5):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        d = agg.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    rows = list(agg.values())
    return rows[skip:] if len(rows) > skip else rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    os.makedirs(a.dst, exist_ok=True)
    shutil.copy(os.path.join(a.src, "trace_kernel_stats.csv"), os.path.join(a.dst, "env_step_kernel_stats.csv"))
    stats = [r for r in csv.DictReader(open(os.path.join(a.src, "trace_kernel_stats.csv"))) if KERNEL in r["Name"]]
    fetch = per_dispatch(os.path.join(a.src, "pmc_FETCH_SIZE_counter_collection.csv"))
    write = per_dispatch(os.path.join(a.src, "pmc_WRITE_SIZE_counter_collection.csv"))
    fk = statistics.mean(d["FETCH_SIZE"] for d in fetch)      # KB per dispatch
    wk = statistics.mean(d["WRITE_SIZE"] for d in write)
    traffic = 2 * fk * 1024 + wk * 1024
    out = {"kernel": stats[0]["Name"] if stats else KERNEL, "envs": a.envs,
           "kernel_avg_ns_rocprof": float(stats[0]["AverageNs"]) if stats else None,
           "dispatches": len(fetch), "fetch_size_kb": fk, "write_size_kb": wk,
           "read_bytes_corrected": 2 * fk * 1024, "write_bytes": wk * 1024,
           "traffic_bytes_per_launch": traffic, "traffic_bytes_per_env_step": traffic / a.envs,
           "note": "FETCH_SIZE doubled (gfx950 reports half of wide coalesced reads); our loads are 4-8 B per "
                   "lane, an uncalibrated width -- the ratio to the algorithmic bytes is the useful number"}
    json.dump(out, open(os.path.join(a.dst, "env_step_pmc_traffic.json"), "w"), indent=1)
    sq = per_dispatch(os.path.join(a.src, "pmc_sq_counter_collection.csv"))
    if sq:
        waves = statistics.mean(d["SQ_WAVES"] for d in sq)
        per_wave = {k: statistics.mean(d[k] for d in sq) / waves for k in sq[0] if k != "SQ_WAVES"}
        json.dump({"kernel": KERNEL, "waves": waves, "per_wave": per_wave,
                   "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are in quad-cycles (x4 = clock cycles)"},
                  open(os.path.join(a.dst, "env_step_sq_counters.json"), "w"), indent=1)
    sq64_path = os.path.join(a.src, "pmc_sq64_counter_collection.csv")
    sq64 = per_dispatch(sq64_path) if os.path.exists(sq64_path) else None
    if sq64:
        waves = statistics.mean(d["SQ_WAVES"] for d in sq64)
        json.dump({"kernel": KERNEL, "waves": waves,
                   "per_wave": {k: statistics.mean(d[k] for d in sq64) / waves for k in sq64[0] if k != "SQ_WAVES"},
                   "note": "fp64 VALU mix per wave, averaged over the kernel's roles (SQ_WAVE_CYCLES / SQ_ACTIVE_* in "
                           "quad-cycles)"},
                  open(os.path.join(a.dst, "env_step_sq_fp64.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
