#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2; do
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-rollout > gpurun_out/kt.$v.json 2> gpurun_out/kt.$v.err || { tail -3 gpurun_out/kt.$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/kt.$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('HIP_FORCE_DEV_KERNARG=$v step %.3f us ev %.3f iso %.3f' % (d['ms_per_step']*1e3, r['kernel_avg_us'], r['isolated_launch_us']))"
done; done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/exp_stamps_split.py --lib tools/st5/c3.so
