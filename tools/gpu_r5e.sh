#!/bin/bash
# Round 5: the whole GPU suite on the in-tree library, then the full bench lines of tools/ab/*.so (tools/ab_full.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -s tests > gpurun_out/r05e_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r05e_pytest.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/r05e_pytest.log | head -20
[ $rc -le 1 ] || exit $rc
ROUNDS=${ROUNDS:-2} timeout -k 10 700 tools/ab_full.sh
