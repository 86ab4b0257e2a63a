#!/bin/bash
# On the GPU box: time each tools/build/ab/<tag>.so (swapped into b747_rl_ctrl_amd/libb747.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
cp b747_rl_ctrl_amd/libb747.so gpurun_out/ab/.orig.so
for round in $(seq ${ROUNDS:-1}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  cp $so b747_rl_ctrl_amd/libb747.so
  timeout -k 10 120 python tools/exp_timing.py --tag $tag > gpurun_out/ab/$tag.txt 2>&1 || { echo "$tag failed rc=$?"; cat gpurun_out/ab/$tag.txt; break; }
  cat gpurun_out/ab/$tag.txt
done
done
cp gpurun_out/ab/.orig.so b747_rl_ctrl_amd/libb747.so
