#!/bin/bash
# On the GPU box: time each tools/build/ab/<tag>.so (loaded through B747_LIB_PATH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for round in $(seq ${ROUNDS:-1}); do
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$PWD/$so
  timeout -k 10 120 python tools/exp_timing.py --tag $tag > gpurun_out/ab/$tag.txt 2>&1 || { echo "$tag failed rc=$?"; cat gpurun_out/ab/$tag.txt; break; }
  cat gpurun_out/ab/$tag.txt
done
done
