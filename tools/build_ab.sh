#!/bin/bash
# Build A/B variants of libb747.so (kernel experiments selected by -D macros) into tools/ab/.
# tools/ab_run.sh loads each through B747_LIB_PATH on the GPU box and times it with tools/exp_timing.py.
cd "$(dirname "$0")/.."
FLAGS=$(python3 -c "import sys; sys.path.insert(0, 'b747_rl_ctrl_amd'); import build; print(' '.join(build.FLAGS))")   # the product's own
build() { tag=$1; shift; /opt/rocm/bin/hipcc $FLAGS "$@" -o tools/ab/$tag.so b747_rl_ctrl_amd/csrc/b747_kernels.hip b747_rl_ctrl_amd/csrc/b747_fast.hip & }
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}
  args=""; for d in ${defs//,/ }; do [ "$d" != "$tag" ] && [ -n "$d" ] && args="$args -D$d"; done
  build $tag $args
done
wait
ls -la tools/ab
