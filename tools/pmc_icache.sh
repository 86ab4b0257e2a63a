#!/bin/bash
# PMC pass on the per-step env kernel: instruction / scalar cache counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-pmc_ic}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQC_DCACHE_MISSES SQC_DCACHE_HITS SQ_WAVES -d $O/prof -o pmc_ic --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || { echo "rc=$?"; tail -3 $O/prof.err; exit 1; }
python3 - "$O/prof" <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_env_step" in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ds = list(agg.values())[5:]
    keys = sorted(ds[0])
    print(f.split("/")[-1], {k: round(sum(d[k] for d in ds) / len(ds), 1) for k in keys}, "(per launch, whole GPU)")
PY
