#!/bin/bash
# On the GPU box: full bench.py line (headline, K-step rollout, PPO rollout, fp32 storage) for each
# tools/ab/<tag>.so loaded through B747_LIB_PATH, ROUNDS times, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/abb; mkdir -p $O
for round in $(seq ${ROUNDS:-1}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$R/$so
  timeout -k 10 180 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/$tag.$round.json 2> $O/$tag.$round.err || { echo "$tag failed"; tail -3 $O/$tag.$round.err; break; }
  python3 - $O/$tag.$round.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:>6s} step {d['ms_per_step']*1e3:6.3f} us ev {r['kernel_avg_us']:6.3f} | rollout {d['rollout']['us_per_step']:6.3f} | ppo {d['ppo_rollout']['us_per_step']:6.3f} | f32 {d['storage_f32']['us_per_step']:6.3f}")
PY
done
done
