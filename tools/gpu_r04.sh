#!/bin/bash
# Round-4 GPU session: full parity suite, bench lines (default and driver arguments), the multi-rank launcher
# rehearsal, rocprofv3 kernel traces and PMC traffic.  Each GPU step under its own timeout; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r04}; O=$R/gpurun_out/$TAG; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -3
  grep -E "FAILED|Error" $O/pytest_gpu.log | head -10
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench_driver_args.err || { tail -5 $O/bench_driver_args.err; exit 1; }
python3 -c "
import json
for f in ('bench.json', 'bench_driver_args.json'):
    d = json.loads(open('$O/' + f).read().strip().splitlines()[-1]); r = d['roofline']
    print(f, d['value'], 'ev', r['kernel_avg_us'], 'frac', r['frac'], 'roll', d['rollout']['us_per_step'], 'ppo', d['ppo_rollout']['us_per_step'],
          'mixed', d['variant_mixed']['step']['us_per_step'], d['variant_mixed']['rollout']['us_per_step'], d['variant_mixed']['ppo_rollout']['us_per_step'],
          'm05', d['sample_time_0.05']['step']['us_per_step'], d['sample_time_0.05']['ppo_rollout']['us_per_step'])"
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_2ranks_gloo.json 2> $O/bench_2ranks_gloo.err || { tail -5 $O/bench_2ranks_gloo.err; exit 1; }
tail -1 $O/bench_2ranks_gloo.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout > $O/bench_under_rocprof.json 2>> $O/prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ppo --output-format csv -- python3 $R/tools/exp_ppo.py 65536 fused > $O/exp_ppo.txt 2>> $O/prof.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/prof -o pmc_$c --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $O/prof -o pmc_sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || echo "sq pmc rc=$?"
find $O/prof -name "*.csv" | head -20
