"""The per-step kernel's time budget (profiles/<round>/env_step_budget.json; bench.py roofline.floor_us) assembled from
that round's committed measurement files, every term citing the file it comes from:
  env_step_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the bench (tools/gpu_prof.sh)
  ubench_budget.txt           the launch-alone and memory-only kernels of the same geometry (tools/ubench_budget.hip)
  stamps.txt                  phase stamps of the -DB747_STAMPS build (tools/exp_stamps_split.py)
  env_step_sq_counters.json   SQ counters per wave, env_step_sq_fp64.json the fp64 VALU mix (tools/pmc_summary.py)
  env_step_pmc_traffic.json   HBM bytes per launch (PMC, tools/pmc_summary.py)
  valu_by_role.json           static VALU per role of the shipped kernel (tools/valu_by_role.py), when present
Usage: python tools/budget_summary.py profiles/r06"""
import csv
import json
import os
import re
import sys

ENVS = 65536
ALGO_B = 277
PEAK_GBS = 8000.0


def main(d):
    rnd = os.path.basename(os.path.normpath(d))
    src = lambda f: f"profiles/{rnd}/{f}"
    terms = {}
    stats = [r for r in csv.DictReader(open(os.path.join(d, "env_step_kernel_stats.csv"))) if "k_env_step_split" in r["Name"]]
    k_us = float(stats[0]["AverageNs"]) / 1e3
    terms["kernel_rocprof_us"] = {"value": round(k_us, 3), "source": src("env_step_kernel_stats.csv"),
                                  "how": f"rocprofv3 --stats average over {stats[0]['Calls']} launches of the bench"}
    ub = {}
    for line in open(os.path.join(d, "ubench_budget.txt")):
        if line.startswith("{"):
            j = json.loads(line)
            ub.setdefault(j["term"], []).append(j["us_per_launch_median"])
    terms["launch_alone_us"] = {"value": round(min(ub["launch"]), 3), "source": src("ubench_budget.txt"),
                                "how": "tools/ubench_budget.hip: 256 x 768-thread workgroups with the per-step kernel's LDS "
                                       "footprint that only pass a barrier, 20 launches per HIP graph, median of 200 replays "
                                       "(dispatch ramp + kernel boundary)"}
    terms["memory_only_us"] = {"value": round(min(ub["memory"]), 3), "source": src("ubench_budget.txt"),
                               "how": "the same geometry loading what each role of the kernel loads for one env step and "
                                      "writing back what it writes (write-through), no arithmetic: launch + the step's HBM "
                                      "traffic in the product's issue order"}
    terms["compute_over_memory_us"] = {"value": round(k_us - min(ub["memory"]), 3),
                                       "how": "kernel_rocprof_us - memory_only_us: what the dependent fp64 work adds to a "
                                              "launch that moves the same bytes"}
    terms["algorithmic_bytes_at_peak_us"] = {"value": round(ALGO_B * ENVS / (PEAK_GBS * 1e3), 3),
                                             "how": "277 B x 65,536 (SURVEY 8(d)) at the 8 TB/s HBM peak"}
    st = open(os.path.join(d, "stamps.txt")).read()
    pct = lambda lab: [float(x) for x in re.search(lab + r" \(us\) percentiles \([^)]*\): ([\d. ]+)", st).group(1).split()]
    starts, barrier, endb = pct("workgroup start"), pct("table barrier"), pct("end - barrier")
    terms["start_spread_us"] = {"value": starts[-1], "source": src("stamps.txt"),
                                "how": "first to last workgroup start (s_memrealtime at each wave's start)"}
    terms["start_to_barrier_us"] = {"value": round(barrier[2] - starts[2], 2), "source": src("stamps.txt"),
                                    "how": "median workgroup: first start to its table barrier (the load phase: the batch's "
                                           "reads and the argument segment arrive)"}
    terms["barrier_to_end_us"] = {"value": endb[2], "source": src("stamps.txt"),
                                  "how": "median workgroup: table barrier to its last wave's end"}
    roles = dict(re.findall(r"(\w+): end - table barrier \(realtime\) median ([\d.]+) us", st))
    terms["role_end_after_barrier_us"] = {"value": {k: float(v) for k, v in roles.items()}, "source": src("stamps.txt"),
                                          "how": "median wave of each role, table barrier to its end"}
    m = re.search(r"deltas posted (\d+)", st)
    if m:
        terms["control_delta_post_cycles"] = {"value": int(m.group(1)), "source": src("stamps.txt"),
                                              "how": "control wave: table barrier to its delta-table post (s_memtime "
                                                     "cycles), which the flight wave's stage 0 waits for"}
    sq = json.load(open(os.path.join(d, "env_step_sq_counters.json")))
    pw, waves = sq["per_wave"], sq["waves"]
    per_simd = waves / 1024.0
    terms["valu_per_env_step"] = {"value": round(pw["SQ_INSTS_VALU"] * 3, 1), "source": src("env_step_sq_counters.json"),
                                  "how": "SQ_INSTS_VALU per wave x 3 waves per env (flight, ahead, control)"}
    terms["valu_busy_frac_simd"] = {"value": round(pw["SQ_ACTIVE_INST_VALU"] * per_simd / pw["SQ_WAVE_CYCLES"], 3),
                                    "source": src("env_step_sq_counters.json"),
                                    "how": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES per wave x waves per SIMD"}
    terms["wait_any_frac_per_wave"] = {"value": round(pw["SQ_WAIT_ANY"] / pw["SQ_WAVE_CYCLES"], 3),
                                       "source": src("env_step_sq_counters.json"), "how": "SQ_WAIT_ANY / SQ_WAVE_CYCLES"}
    f64 = json.load(open(os.path.join(d, "env_step_sq_fp64.json")))["per_wave"]
    terms["fp64_valu_per_env_step"] = {"value": round(3 * sum(v for k, v in f64.items() if k.endswith("_F64")), 1),
                                       "source": src("env_step_sq_fp64.json"),
                                       "how": "3 waves x SQ_INSTS_VALU_{ADD,FMA,MUL,TRANS}_F64 per wave"}
    vr = os.path.join(d, "valu_by_role.json")
    if os.path.exists(vr):
        v = json.load(open(vr))
        terms["valu_per_env_step_by_role_static"] = {
            "value": {k: v["valu"][k] for k in ("flight", "ahead", "control")},
            "v_cndmask": {k: v["v_cndmask"][k] for k in ("flight", "ahead", "control")},
            "source": src("valu_by_role.json"),
            "how": "static VALU of each role's path in the gfx950 listing (tools/valu_by_role.py; the reset path apart)"}
    tr = json.load(open(os.path.join(d, "env_step_pmc_traffic.json")))
    terms["hbm_traffic_bytes_per_env_step"] = {"value": round(tr["traffic_bytes_per_env_step"], 1),
                                               "source": src("env_step_pmc_traffic.json"),
                                               "how": "PMC FETCH_SIZE x 2 (gfx950) + WRITE_SIZE per launch / 65,536"}
    out = {"kernel": "k_env_step_split<double, false> (FAST fp64, b747_env_step, 65,536 envs, one env step per launch)",
           "round": rnd, "terms": terms,
           "reading": (f"a launch that only moves the step's bytes takes {min(ub['memory']):.2f} us ({min(ub['launch']):.2f} of "
                       f"it the launch alone); the kernel takes {k_us:.2f}: the fp64 work adds "
                       f"{k_us - min(ub['memory']):.2f} us on top of the memory-bound launch. Its reads land in one burst at "
                       f"the start (start -> barrier {barrier[2] - starts[2]:.2f} us), its writes in one at the end; "
                       f"between them the three waves of each SIMD issue VALU "
                       f"{terms['valu_busy_frac_simd']['value']:.0%} of the launch's cycles")}
    json.dump(out, open(os.path.join(d, "env_step_budget.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r06")
