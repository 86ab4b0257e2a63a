#!/bin/bash
# Round-5 GPU call: parity of the in-tree library, the A/B of tools/ab/*.so, parity of the ahead-wave build, stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTESTS="tests/test_gpu_tb_pin.py::test_gpu_bench_kernels_reproduce_the_recorded_step_tests tests/test_gpu_mixed.py tests/test_gpu_episode_replay.py tests/test_abi.py" \
  ROUNDS=3 NOPROF=1 tools/gpu_ab.sh || exit $?
cp b747_rl_ctrl_amd/libb747.so gpurun_out/.orig.so
cp tools/ab/r3.so b747_rl_ctrl_amd/libb747.so
timeout -k 10 400 python -u -m pytest --maxfail=10 -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_tb_pin.py::test_gpu_bench_kernels_reproduce_the_recorded_step_tests tests/test_gpu_episode_replay.py tests/test_gpu_fullsize.py \
  > gpurun_out/r3_pytest.log 2>&1; rc=$?
cp gpurun_out/.orig.so b747_rl_ctrl_amd/libb747.so
echo "r3 pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3_pytest.log | tail -2; grep -E "FAILED" gpurun_out/r3_pytest.log | head
[ $rc -le 1 ] || exit $rc
echo "== stamps r2"; timeout -k 10 120 python tools/exp_stamps_split.py --lib tools/st5/r2.so || exit 1
echo "== stamps r3"; timeout -k 10 120 python tools/exp_stamps_split.py --lib tools/st5/r3.so --roles 3
