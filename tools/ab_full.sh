#!/bin/bash
# On the GPU box: the full bench line (headline per-step kernel, K = 100 rollout, config-5 PPO rollout, MIXED) of each
# ${AB_DIR:-tools/ab}/<tag>.so loaded through B747_LIB_PATH, ROUNDS times interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/abf; mkdir -p $O
for round in $(seq ${ROUNDS:-2}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$R/$so
  timeout -k 10 180 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/$tag.$round.json 2> $O/$tag.$round.err || { echo "$tag failed"; tail -3 $O/$tag.$round.err; exit 1; }
  python3 - $O/$tag.$round.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
g = lambda k, f: (d.get(k) or {}).get(f)
m, s5 = d.get("variant_mixed") or {}, d.get("sample_time_0.05") or {}
print(f"{sys.argv[2]:>10s} step ev {r['kernel_avg_us']:7.3f} us | rollout {g('rollout', 'us_per_step')} | ppo {g('ppo_rollout', 'us_per_step')} "
      f"| mixed step {(m.get('step') or {}).get('us_per_step')} roll {(m.get('rollout') or {}).get('us_per_step')} "
      f"ppo {(m.get('ppo_rollout') or {}).get('us_per_step')} | st0.05 step {(s5.get('step') or {}).get('us_per_step')} "
      f"roll {(s5.get('rollout') or {}).get('us_per_step')} ppo {(s5.get('ppo_rollout') or {}).get('us_per_step')}", flush=True)
PY
done
done
