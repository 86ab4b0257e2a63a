#!/bin/bash
# Round-end GPU check without profilers: the full parity suite, the bench lines (default and driver arguments)
# and the two-rank launcher rehearsal.  Each GPU step under its own timeout; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r06}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -3
grep -E "FAILED|Error" $O/pytest_gpu.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench_driver_args.err || { tail -5 $O/bench_driver_args.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_2ranks_gloo.json 2> $O/bench_2ranks_gloo.err || { tail -5 $O/bench_2ranks_gloo.err; exit 1; }
python3 -c "
import json
for f in ('bench.json', 'bench_driver_args.json', 'bench_2ranks_gloo.json'):
    d = json.loads(open('$O/' + f).read().strip().splitlines()[-1]); r = d['roofline']
    print(f, d['value'], d['ms_per_step'], 'ev', r['kernel_avg_us'], 'frac', r['frac'], 'ranks', d['ranks_seen'])
    for k in ('rollout', 'ppo_rollout', 'ppo_training'):
        if d.get(k): print('  ', k, d[k].get('value'), d[k].get('us_per_step', d[k].get('s_per_iteration')))"
