#!/bin/bash
# Build A/B variants of libb747.so that differ in compiler flags: "tag|extra flags" per argument,
# into tools/ab/ (tools/ab_run.sh times each on the GPU box).
cd "$(dirname "$0")/.."
mkdir -p tools/ab
FLAGS="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-machine-licm -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=14"
for spec in "$@"; do
  tag=${spec%%|*}; extra=${spec#*|}
  /opt/rocm/bin/hipcc $FLAGS $extra -o tools/ab/$tag.so b747_rl_ctrl_amd/csrc/b747_kernels.hip b747_rl_ctrl_amd/csrc/b747_fast.hip &
done
wait
ls -la tools/ab
