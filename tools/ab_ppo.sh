#!/bin/bash
# On the GPU box: config-5 rollout timing (fused and two-launch) for each tools/ab/<tag>.so
# loaded through B747_LIB_PATH.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  for mode in fused split; do
    timeout -k 10 120 python tools/exp_ppo.py 65536 $tag-$mode > gpurun_out/ab/ppo_$tag-$mode.txt 2>&1 || { echo "$tag failed rc=$?"; cat gpurun_out/ab/ppo_$tag-$mode.txt; exit 1; }
    grep "graph=True" gpurun_out/ab/ppo_$tag-$mode.txt
  done
done
