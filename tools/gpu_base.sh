#!/bin/bash
# Round-5 baseline on the GPU box: the default bench line and a rocprofv3 kernel-trace of the per-step bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r05base}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout --steps 400 > $O/bench_prof.json 2> $O/bench_prof.err) || { tail -5 $O/bench_prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200
tail -1 $O/bench.json | cut -c1-1500
