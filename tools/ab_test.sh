#!/bin/bash
# On the GPU box: run one pytest selection against each ${AB_DIR:-tools/ab}/*.so (loaded through B747_LIB_PATH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abt
for so in ${AB_DIR:-tools/ab}/*.so; do
  tag=$(basename $so .so)
  export B747_LIB_PATH=$(realpath $so)
  timeout -k 10 ${AB_TIMEOUT:-300} python -u -m pytest -x -q --timeout 250 --timeout-method thread "$@" > gpurun_out/abt/$tag.txt 2>&1
  rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/abt/$tag.txt)"
  case $rc in 0|1) ;; *) break ;; esac
done
