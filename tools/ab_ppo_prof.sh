#!/bin/bash
# On the GPU box: rocprofv3 kernel-trace averages of the config-5 kernels (k_ppo_rollout, k_policy_value) in
# tools/exp_ppo.py's fused rollouts, for each ${AB_DIR:-tools/ab}/<tag>.so loaded through B747_LIB_PATH.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/abpp
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abpp/$tag -o t --output-format csv -- python3 $R/tools/exp_ppo.py 65536 $tag-fused > $R/gpurun_out/abpp/$tag.txt 2>&1) || { echo "$tag failed"; tail -3 gpurun_out/abpp/$tag.txt; break; }
  grep "graph=True" gpurun_out/abpp/$tag.txt
  python3 - "$R/gpurun_out/abpp/$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_ppo_rollout" in r["Name"] or "k_rollout_split<true" in r["Name"] or "k_policy_value" in r["Name"]:
        nm = "k_ppo_rollout" if "rollout" in r["Name"] else "k_policy_value"
        avg = float(r["AverageNs"]) / 1e3
        print(f"{sys.argv[2]:>10s} {nm:>15s} calls {r['Calls']:>4s} avg {avg:9.2f} us = {avg / 64:6.3f} us per rollout step")
PY
done
