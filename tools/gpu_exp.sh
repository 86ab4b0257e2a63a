#!/bin/bash
# On the GPU box: one experiment session.  Each GPU step has its own time limit; the script stops at
# the first failure.  Env: TAG (output dir under gpurun_out/), TESTS (pytest selection, "" = skip),
# STAMPS=1 (phase stamps from tools/st/*.so), AB=1 (rocprof + timing probe of tools/ab/*.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-exp}; O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$STAMPS" ]; then
  if [ -f tools/st/stamps.so ]; then
    timeout -k 10 120 python tools/exp_stamps.py --lib tools/st/stamps.so > $O/st_phase.txt 2>&1 || { cat $O/st_phase.txt; exit 1; }
    grep -v amdgpu.ids $O/st_phase.txt
  fi
  if [ -f tools/st/stamps_step.so ]; then
    timeout -k 10 120 python tools/exp_stamps.py --lib tools/st/stamps_step.so --step > $O/st_step.txt 2>&1 || { cat $O/st_step.txt; exit 1; }
    grep -v amdgpu.ids $O/st_step.txt
  fi
fi
if [ -n "$AB" ]; then
  ROUNDS=${ROUNDS:-2} bash tools/ab_prof.sh || exit $?
  ROUNDS=1 bash tools/ab_run.sh || exit $?
fi
