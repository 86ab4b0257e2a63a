#!/bin/bash
# On the GPU box: rocprof kernel stats of the config-5 rollout for each tools/build/ab/<tag>.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/abppo
cp b747_rl_ctrl_amd/libb747.so gpurun_out/abppo/.orig.so
for so in tools/build/ab/*.so; do
  tag=$(basename $so .so)
  cp $so b747_rl_ctrl_amd/libb747.so
  (cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abppo/$tag -o p --output-format csv -- python3 $R/tools/exp_ppo.py 65536 $tag > $R/gpurun_out/abppo/$tag.txt 2>&1) || { echo "$tag failed"; break; }
  grep "graph=True" gpurun_out/abppo/$tag.txt
  python3 -c "import csv,glob;r=[x for x in csv.DictReader(open(glob.glob('$R/gpurun_out/abppo/$tag/**/*kernel_stats.csv',recursive=True)[0])) if 'policy' in x['Name']];print('$tag policy ns', r[0]['AverageNs'])"
done
cp gpurun_out/abppo/.orig.so b747_rl_ctrl_amd/libb747.so
