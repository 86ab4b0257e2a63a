#!/bin/bash
# Round-3 diagnostics on the GPU box: quick A/B of tools/ab/*.so, then phase stamps of each tools/st/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/diag
if [ -z "$SKIP_AB" ]; then ROUNDS=${ROUNDS:-3} bash tools/ab_quick.sh || exit 1; fi
for so in tools/st/*.so; do
  tag=$(basename $so .so)
  timeout -k 10 120 python -u tools/exp_stamps_split.py --lib $so > gpurun_out/diag/$tag.txt 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/diag/$tag.txt; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids gpurun_out/diag/$tag.txt
done
