#!/bin/bash
# On the GPU box: the GPU test suite, then the env-step phase stamps (diagnostic build
# tools/st/stamps_step.so) for 1- and 2-step launches, then the A/B builds in tools/ab/
# (rocprof durations + timing probe).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -f tools/st/stamps_step.so ]; then
  for k in 1 2; do
    timeout -k 10 120 python tools/exp_stamps.py --lib tools/st/stamps_step.so --k $k --step > gpurun_out/st_step$k.txt 2>&1 || exit $?
    grep -v amdgpu.ids gpurun_out/st_step$k.txt
  done
fi
if ls tools/ab/*.so > /dev/null 2>&1; then
  ROUNDS=${ROUNDS:-2} bash tools/ab_prof.sh || exit $?
  ROUNDS=1 bash tools/ab_run.sh || exit $?
fi
