#!/bin/bash
# A/B of the per-step kernel's split read-out (B747_RO_SPLIT): parity of the variant (the split-kernel equality tests
# and the tk = 20 s oracle replay of the per-step kernel with its library swapped in), then interleaved timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abro; mkdir -p $O
cp b747_rl_ctrl_amd/libb747.so $O/.orig.so
cp tools/ab/g_rosplit.so b747_rl_ctrl_amd/libb747.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split.py \
  "tests/test_gpu_episode_replay.py::test_bench_kernel_tk20_episode_every_env_every_step" > $O/pytest_rosplit.log 2>&1; rc=$?
cp $O/.orig.so b747_rl_ctrl_amd/libb747.so
tail -3 $O/pytest_rosplit.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash tools/ab_quick.sh
