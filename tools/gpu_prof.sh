#!/bin/bash
# Profile session: rocprofv3 kernel traces (per-step bench, config-5 rollout), PMC passes (HBM bytes, SQ counters,
# fp64 VALU mix) of the per-step kernel, phase stamps of a -DB747_STAMPS build (tools/st/stamps.so: tools/build_stamps.sh)
# and the launch / memory terms (tools/ub/ubench_budget).  Summaries: tools/pmc_summary.py, tools/budget_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-r06prof}; mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout > $O/prof_trace_bench.json 2>> $O/prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ppo --output-format csv -- python3 $R/tools/exp_ppo.py 65536 fused > $O/exp_ppo.txt 2>> $O/prof.err || exit $?
grep graph $O/exp_ppo.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/prof -o pmc_$c --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $O/prof -o pmc_sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/prof -o pmc_sq64 --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2>> $O/prof.err || exit $?
cd $R
timeout -k 10 120 python tools/exp_stamps_split.py --lib tools/st/stamps.so > $O/stamps.txt 2>&1 || exit 1
cat $O/stamps.txt
timeout -k 10 120 tools/ub/ubench_budget > $O/ubench_budget.txt 2>&1 || exit 1
cat $O/ubench_budget.txt
find $O/prof -name "*.csv" | head -30
