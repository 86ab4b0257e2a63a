#!/bin/bash
# One GPU-box session: parity tests, bench lines, kernel timing experiment, rocprofv3 kernel
# trace + separate PMC passes.  Everything lands in gpurun_out/; copy what is judged to profiles/.
# Each GPU step runs under its own timeout and the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r01c}; O=$R/gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
for extra in "--variant faithful" "--x32" "--eager"; do
  name=$(echo $extra | tr -d ' -')
  timeout -k 10 200 python bench.py $extra --no-cpu-baseline > $O/bench_$name.json 2>> $O/bench.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
timeout -k 10 200 python tools/exp_timing.py > $O/exp_timing.txt 2>&1 || exit $?
cat $O/exp_timing.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout > $O/prof_trace_bench.json 2>> $O/prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ppo --output-format csv -- python3 $R/tools/exp_ppo.py 65536 fused > $O/exp_ppo.txt 2>> $O/prof.err || exit $?
grep graph $O/exp_ppo.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $O/prof -o pmc_$c --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $O/prof -o pmc_sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || echo "sq pmc failed rc=$?"
find $O/prof -name "*.csv" | head -20
