#!/bin/bash
# Round 6: stamps of tools/st/*.so, rocprof A/B of the per-step kernel and of the config-5 kernels for tools/ab/*.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOQUICK=1 PROF_ROUNDS=${PROF_ROUNDS:-3} bash tools/gpu_r6f.sh || exit $?
for r in 1 2; do timeout -k 10 900 bash tools/ab_ppo_prof.sh || exit $?; done
