#!/bin/bash
# bench variants + rocprof kernel trace + PMC (FETCH_SIZE / WRITE_SIZE in separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/prof
R=$PWD
TAG=${TAG:-r01}
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
timeout -k 10 200 python bench.py --eager --no-cpu-baseline > gpurun_out/bench_${TAG}_eager.json 2>>gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 200 python bench.py --x32 --no-cpu-baseline > gpurun_out/bench_${TAG}_x32.json 2>>gpurun_out/bench_$TAG.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/$TAG -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_trace_$TAG.json 2>>$R/gpurun_out/prof_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof/$TAG -o pmc_fetch --output-format csv -- python3 $R/bench.py --eager --steps 40 --warmup 5 --no-cpu-baseline > /dev/null 2>>$R/gpurun_out/prof_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof/$TAG -o pmc_write --output-format csv -- python3 $R/bench.py --eager --steps 40 --warmup 5 --no-cpu-baseline > /dev/null 2>>$R/gpurun_out/prof_$TAG.err || exit $?
find $R/gpurun_out/prof/$TAG -name '*.csv' | head -20
cat $R/gpurun_out/bench_${TAG}_eager.json $R/gpurun_out/bench_${TAG}_x32.json
