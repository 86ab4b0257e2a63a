#!/bin/bash
# On the GPU box: the headline bench line only (--no-rollout) for each ${AB_DIR:-tools/ab}/<tag>.so loaded through B747_LIB_PATH,
# ROUNDS times interleaved; prints the launch period and the timed-region event time per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/abq; mkdir -p $O
for round in $(seq ${ROUNDS:-2}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-rollout ${BENCH_ARGS} > $O/$tag.$round.json 2> $O/$tag.$round.err || { echo "$tag failed"; tail -3 $O/$tag.$round.err; exit 1; }
  python3 - $O/$tag.$round.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:>10s} step {d['ms_per_step']*1e3:7.3f} us  ev {r['kernel_avg_us']:7.3f} us  iso {r['isolated_launch_us']:7.3f}", flush=True)
PY
done
done
