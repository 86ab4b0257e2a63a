#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace.  Stops at the first GPU fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
STEPS=${STEPS:-400}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 20 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err
rc=$?; echo "rocprof rc=$rc"; find $R/gpurun_out/prof -name '*stats*' | head
exit $rc
