#!/bin/bash
# Round 5: A/B of tools/ab/*.so (headline line), stamps of tools/st5/*.so, parity of ${TEST_SO} (per-step kernel tests).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} NOPROF=1 tools/gpu_ab.sh || exit $?
for so in $(ls tools/st5/*.so 2>/dev/null); do echo "== stamps $so"; timeout -k 10 120 python tools/exp_stamps_split.py --lib $so | grep -E 'flight|control|ahead|realtime' || exit 1; done
if [ -n "$TEST_SO" ]; then
  cp b747_rl_ctrl_amd/libb747.so gpurun_out/.orig_t.so
  cp $TEST_SO b747_rl_ctrl_amd/libb747.so
  timeout -k 10 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_episode_replay.py::test_bench_kernel_tk20_episode_every_env_every_step tests/test_gpu_vec_env.py tests/test_gpu_episode_stats.py tests/test_gpu_tb_pin.py::test_gpu_bench_kernels_reproduce_the_recorded_step_tests tests/test_gpu_fullsize.py > gpurun_out/t_pytest.log 2>&1; rc=$?
  cp gpurun_out/.orig_t.so b747_rl_ctrl_amd/libb747.so
  echo "test pytest rc=$rc"; grep -E "passed|failed" gpurun_out/t_pytest.log | tail -1; grep -E "^FAILED" gpurun_out/t_pytest.log | head
fi
