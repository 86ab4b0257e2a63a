#!/bin/bash
# Round-5 GPU call: parity of the in-tree library (three-role per-step kernel), A/B of tools/ab/*.so, stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTESTS="tests/test_gpu_tb_pin.py::test_gpu_bench_kernels_reproduce_the_recorded_step_tests tests/test_gpu_mixed.py::test_mixed_free_running_episode_against_fast_and_the_oracle tests/test_gpu_episode_replay.py tests/test_gpu_fullsize.py tests/test_gpu_env.py" \
  ROUNDS=3 NOPROF=1 tools/gpu_ab.sh || exit $?
for so in tools/st5/*.so; do echo "== stamps $so"; timeout -k 10 120 python tools/exp_stamps_split.py --lib $so || exit 1; done
