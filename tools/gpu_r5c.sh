#!/bin/bash
# A/B of tools/ab/*.so (headline line), then stamps of tools/st5/*.so; optional PYTESTS first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} NOPROF=1 tools/gpu_ab.sh || exit $?
for so in tools/st5/*.so; do echo "== stamps $so"; timeout -k 10 120 python tools/exp_stamps_split.py --lib $so || exit 1; done
