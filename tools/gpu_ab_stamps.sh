#!/bin/bash
# Phase stamps of every tools/st/*.so (tools/exp_stamps_split.py), then tools/gpu_ab.sh (optional PYTESTS on PYTEST_LIB,
# the rocprofv3 A/B of tools/ab/*.so over PROF_ROUNDS interleaved rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/st
for so in tools/st/*.so; do
  t=$(basename $so .so)
  timeout -k 10 120 python3 tools/exp_stamps_split.py --lib $so > gpurun_out/st/$t.txt 2>&1 || { tail -5 gpurun_out/st/$t.txt; exit 1; }
  echo "== $t"; head -4 gpurun_out/st/$t.txt
done
NOQUICK=1 PROF_ROUNDS=${PROF_ROUNDS:-3} bash tools/gpu_ab.sh
