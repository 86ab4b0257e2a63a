#!/bin/bash
# Build A/B variants of libb747.so that differ in compiler flags: "tag|extra flags" per argument,
# into tools/ab/ (tools/ab_run.sh times each on the GPU box).
cd "$(dirname "$0")/.."
mkdir -p tools/ab
FLAGS=$(python3 -c "import sys; sys.path.insert(0, 'b747_rl_ctrl_amd'); import build; print(' '.join(build.FLAGS))")   # the product's own
for spec in "$@"; do
  tag=${spec%%|*}; extra=${spec#*|}
  /opt/rocm/bin/hipcc $FLAGS $extra -o tools/ab/$tag.so b747_rl_ctrl_amd/csrc/b747_kernels.hip b747_rl_ctrl_amd/csrc/b747_fast.hip &
done
wait
ls -la tools/ab
