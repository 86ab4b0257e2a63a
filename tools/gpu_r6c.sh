#!/bin/bash
# Round 6: the GPU suite on the theta-in-ahead build, the per-step kernel A/B (rocprof), config 2 per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/c2
PYTESTS=tests PYTEST_LIB=tools/ab/b_tha.so NOQUICK=1 PROF_ROUNDS=3 bash tools/gpu_ab.sh || exit $?
for so in tools/ab/*.so; do
  B747_LIB_PATH=$R/$so timeout -k 10 120 python3 -u tools/exp_config2.py 2 > gpurun_out/c2/$(basename $so .so).txt 2>&1 || { tail -5 gpurun_out/c2/$(basename $so .so).txt; exit 1; }
  cat gpurun_out/c2/$(basename $so .so).txt
done
