#!/bin/bash
# The HIP runtime's graph-launch knobs against the short timed region (bench.py --steps 20) and the host cost of
# hipGraphLaunch (tools/exp_k20.py).  One bench run per setting, each under its own timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/graphflags; mkdir -p $O
for spec in "default:" "pc0:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "pc1:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" \
            "bs1:DEBUG_HIP_GRAPH_BATCH_SIZE=1" "bs8:DEBUG_HIP_GRAPH_BATCH_SIZE=8" "bs32:DEBUG_HIP_GRAPH_BATCH_SIZE=32"; do
  tag=${spec%%:*}; kv=${spec#*:}
  for K in 20 400; do
    env $kv timeout -k 10 120 python3 -u bench.py --steps $K --warmup 5 --no-rollout --no-cpu-baseline > $O/$tag.$K.json 2> $O/$tag.$K.err || { echo "$tag $K failed"; tail -3 $O/$tag.$K.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/$tag.$K.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$tag', $K, 'us/step', round(d['ms_per_step']*1e3,3), 'ev', r['kernel_avg_us'])"
  done
  env $kv timeout -k 10 120 python3 -u tools/exp_k20.py 20 2>/dev/null | grep -E "replay 2|host" | head -4
done
