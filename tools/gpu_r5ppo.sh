#!/bin/bash
# Round 5: config-5 rollout A/B (tools/ab/*.so: fused-rollout timing + rocprof kernel averages, tools/ab_ppo_prof.sh),
# then the PPO parity tests with ${PPO_TEST_SO} swapped in.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do AB_DIR=tools/ab timeout -k 10 600 bash tools/ab_ppo_prof.sh || exit 1; done
if [ -n "$PPO_TEST_SO" ]; then
  cp b747_rl_ctrl_amd/libb747.so gpurun_out/.orig_ppo.so
  cp $PPO_TEST_SO b747_rl_ctrl_amd/libb747.so
  timeout -k 10 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_ppo.py tests/test_gpu_episode_replay.py::test_ppo_rollout_kernel_tk20_episode_every_env_every_step "tests/test_gpu_mixed.py::test_mixed_ppo_rollout_kernel_per_step_parity" tests/test_gpu_tb_pin.py > gpurun_out/ppo_pytest.log 2>&1; rc=$?
  cp gpurun_out/.orig_ppo.so b747_rl_ctrl_amd/libb747.so
  echo "ppo pytest rc=$rc"; grep -E "passed|failed" gpurun_out/ppo_pytest.log | tail -1; grep -E "^FAILED" gpurun_out/ppo_pytest.log | head
fi
