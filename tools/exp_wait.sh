#!/bin/bash
# The driver's short timed region (--steps 20) against the HIP runtime's host wait for completion: the default
# against ROC_ACTIVE_WAIT_TIMEOUT (us of active polling before an interrupt wait), ROUNDS interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wait; mkdir -p $O
for r in $(seq ${ROUNDS:-3}); do
for w in default 50 1000; do
  if [ $w = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$w; fi
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-rollout --no-cpu-baseline > $O/$w.$r.json 2> $O/$w.$r.err || { tail -3 $O/$w.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$w.$r.json').read().strip().splitlines()[-1]);print('$w', d['value'], d['ms_per_step']*1e3, 'ev', d['roofline']['kernel_avg_us'])"
done; done
