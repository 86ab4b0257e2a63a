#!/bin/bash
# On the GPU box: SQ counters (one --pmc pass) of the env-step kernel for each ${AB_DIR:-tools/ab}/<tag>.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/absq
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/absq/$tag -o sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2> $R/gpurun_out/absq/$tag.err) || { echo "$tag failed"; tail -3 gpurun_out/absq/$tag.err; break; }
  python3 - "$R/gpurun_out/absq/$tag" "$tag" <<'PY'
import collections, csv, glob, statistics, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    if "k_env_step" not in r["Kernel_Name"]:
        continue
    agg.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
rows = list(agg.values())[5:]
w = statistics.mean(d["SQ_WAVES"] for d in rows)
print(sys.argv[2], f"waves {w:.0f} per-wave:", ", ".join(f"{k[3:]} {statistics.mean(d[k] for d in rows) / w:.0f}" for k in rows[0] if k != "SQ_WAVES"))
PY
done
