#!/bin/bash
# Round 6: max-ilp scheduler A/B (rocprof per-step kernel, full bench lines), then the GPU suite on the max-ilp build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=3 tools/ab_prof.sh || exit 1
ROUNDS=2 tools/ab_full.sh || exit 1
export B747_LIB_PATH=$PWD/tools/ab/maxilp.so
timeout -k 10 800 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests > gpurun_out/r06a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r06a_pytest.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/r06a_pytest.log | head -20
exit $rc
