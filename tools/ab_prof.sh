#!/bin/bash
# On the GPU box: rocprofv3 kernel-trace average of k_env_steps for each tools/ab/<tag>.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/abp
for round in $(seq ${ROUNDS:-1}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$R/$so
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abp/$tag.$round -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout --steps 400 > $R/gpurun_out/abp/$tag.$round.json 2> $R/gpurun_out/abp/$tag.$round.err) || { echo "$tag failed"; tail -3 gpurun_out/abp/$tag.$round.err; break; }
  python3 - "$R/gpurun_out/abp/$tag.$round" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_env_step" in r["Name"]:
        print(f"{sys.argv[2]:>8s} k_env_steps calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:7.3f} us min {float(r['MinNs'])/1e3:7.3f} max {float(r['MaxNs'])/1e3:7.3f}")
PY
done
done
