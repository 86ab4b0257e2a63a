#!/bin/bash
# On the GPU box: SQ counters of the fused config-5 rollout kernel (k_ppo_rollout), one --pmc pass
# (8 SQ counters, the set tools/gpu_r02.sh uses for the env-step kernel) over tools/exp_ppo.py.
# Summary: python tools/pmc_ppo_summary.py gpurun_out/<TAG>/prof profiles/r02
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-ppo_sq}; O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $O/prof -o pmc_sq --output-format csv -- python3 $R/tools/exp_ppo.py 65536 fused > $O/exp_ppo_pmc.txt 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cat $O/exp_ppo_pmc.txt
find $O/prof -name "*.csv"
