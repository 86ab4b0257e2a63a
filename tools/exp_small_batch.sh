#!/bin/bash
# Small-batch timing of the per-step, K-step and PPO-rollout paths for each tools/ab/<tag>.so (B747_LIB_PATH):
# bench.py at --envs N (its headline per-step line and the K = 100 rollout line) and tools/exp_ppo.py N fused.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/small; mkdir -p $O
for n in ${SIZES:-4096 16384}; do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  timeout -k 10 200 python3 -u bench.py --envs $n --no-cpu-baseline --no-main05 --steps 100 > $O/$tag.$n.json 2> $O/$tag.$n.err || { echo "$tag $n failed"; tail -3 $O/$tag.$n.err; exit 1; }
  python3 - $O/$tag.$n.json $tag $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rollout") or {}
print(f"{sys.argv[2]:>8s} n={sys.argv[3]:>6s} step {d['roofline']['kernel_avg_us']:7.3f} us  rollout {r.get('us_per_step')} us/step", flush=True)
PY
  timeout -k 10 120 python3 tools/exp_ppo.py $n fused 2>/dev/null | grep "graph=True" | sed "s/^/$tag n=$n ppo /"
done
done
