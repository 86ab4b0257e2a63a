#!/bin/bash
# A/B on the GPU box: optional parity tests of the in-tree library first (PYTESTS), then the headline bench line of
# every tools/ab/*.so (ab_quick, ROUNDS interleaved; NOQUICK skips it) and a rocprofv3 kernel-trace average of each
# (ab_prof, PROF_ROUNDS interleaved; NOPROF skips it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
if [ -n "$PYTESTS" ]; then
  # PYTEST_LIB: run the tests on that A/B build instead of the in-tree library
  B747_LIB_PATH=${PYTEST_LIB:+$R/$PYTEST_LIB} timeout -k 10 600 python -u -m pytest --maxfail=10 -v -s --timeout 240 --timeout-method thread -m gpu $PYTESTS > gpurun_out/ab_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/ab_pytest.log | tail -2; grep -E "FAILED|Error|assert" gpurun_out/ab_pytest.log | head -20
  # rc 1 = assertion failures (keep going to the A/B); anything else (timeout, abort, fault) ends the call
  [ $rc -le 1 ] || exit $rc
fi
[ -n "$NOQUICK" ] || ROUNDS=${ROUNDS:-3} timeout -k 10 600 tools/ab_quick.sh || exit 1
[ -n "$NOPROF" ] || ROUNDS=${PROF_ROUNDS:-1} timeout -k 10 900 tools/ab_prof.sh
