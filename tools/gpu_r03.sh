#!/bin/bash
# Round-3 GPU session: parity tests, bench line, rocprofv3 kernel trace + separate PMC passes.
# Every GPU step runs under its own timeout; the script stops at the first failure.
# Env: TAG (output dir under gpurun_out/), SKIP_TESTS=1, TESTS="tests/..." (subset), SKIP_PMC=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r03final}; O=$R/gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_args.json 2>> $O/bench.err || exit 1
cat $O/bench_driver_args.json
[ -n "$SKIP_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout > $O/prof_trace_bench.json 2>> $O/prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ppo --output-format csv -- python3 $R/tools/exp_ppo.py 65536 fused > $O/exp_ppo.txt 2>> $O/prof.err || exit 1
[ -n "$SKIP_PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/prof -o pmc_$c --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $O/prof -o pmc_sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit 1
find $O/prof -name "*.csv" | head -20
