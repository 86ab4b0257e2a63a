#!/bin/bash
# On the GPU box: the bench's secondary lines (K = 100 rollout, config-5 PPO) for each tools/ab/<tag>.so
# loaded through B747_LIB_PATH. ROUNDS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abr
for round in $(seq ${ROUNDS:-1}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/abr/$tag.$round.json 2> gpurun_out/abr/$tag.$round.err || { echo "$tag failed"; tail -3 gpurun_out/abr/$tag.$round.err; break; }
  python3 -c "import json; d = json.loads(open('gpurun_out/abr/$tag.$round.json').read().splitlines()[-1]); print(f\"{'$tag':>10s} rollout {d['rollout']['us_per_step']:.3f} us/step  ppo {d['ppo_rollout']['us_per_step']:.3f}  step {d['roofline']['kernel_avg_us']:.3f}\")"
done
done
