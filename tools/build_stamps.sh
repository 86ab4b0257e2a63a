#!/bin/bash
# The diagnostic build of the per-step kernel's phase stamps (-DB747_STAMPS, b747_lanes.h) with the product's flags, into
# tools/st/stamps.so (tools/exp_stamps_split.py, tools/exp_stamps_ppo.py), and the budget microbenchmark tools/ub/ubench_budget.
cd "$(dirname "$0")/.."
mkdir -p tools/st tools/ub
FLAGS=$(python3 -c "import sys; sys.path.insert(0, 'b747_rl_ctrl_amd'); import build; print(' '.join(build.FLAGS))")
/opt/rocm/bin/hipcc $FLAGS -DB747_STAMPS -o tools/st/stamps.so b747_rl_ctrl_amd/csrc/b747_kernels.hip b747_rl_ctrl_amd/csrc/b747_fast.hip &
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o tools/ub/ubench_budget tools/ubench_budget.hip &
wait
ls -la tools/st tools/ub
