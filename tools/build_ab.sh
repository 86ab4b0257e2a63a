#!/bin/bash
# Build A/B variants of libb747.so (kernel experiments selected by -D macros) into tools/ab/.
# tools/ab_run.sh swaps each into place on the GPU box and times it with tools/exp_timing.py.
cd "$(dirname "$0")/.."
FLAGS="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-machine-licm -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=14"
build() { tag=$1; shift; /opt/rocm/bin/hipcc $FLAGS "$@" -o tools/ab/$tag.so b747_rl_ctrl_amd/csrc/b747_kernels.hip b747_rl_ctrl_amd/csrc/b747_fast.hip & }
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}
  args=""; for d in ${defs//,/ }; do [ "$d" != "$tag" ] && [ -n "$d" ] && args="$args -D$d"; done
  build $tag $args
done
wait
ls -la tools/ab
