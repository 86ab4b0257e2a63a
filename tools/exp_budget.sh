#!/bin/bash
# Speed-of-light budget of the per-step kernel (k_env_step_split) on the GPU box (bench.py roofline.floor):
#  1. per-launch time in the bench's HIP graph for the shipping build and two diagnostic builds of the same source:
#     B747_DIAG_MEM=1 (the launch alone: dispatch ramp + kernel boundary), =2 (+ this kernel's loads and stores);
#  2. phase stamps of a -DB747_STAMPS build (in-wave timeline: prologue, stages, tail);
#  3. SQ counters of the shipping kernel (VALU issue, fp64 VALU mix) in their own --pmc pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-budget}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mixed.py > $O/pytest_mixed.log 2>&1; echo "mixed tests rc=$?"; grep -E "PASS|FAIL|worst|Error" $O/pytest_mixed.log | head -20
ROUNDS=${ROUNDS:-3} bash tools/ab_quick.sh > $O/ab_quick.txt 2>&1 || { cat $O/ab_quick.txt; exit 1; }
cat $O/ab_quick.txt
for v in fast mixed; do
  timeout -k 10 200 python3 tools/exp_mixed_parity.py --variant $v > $O/parity_$v.txt 2>&1 || { tail -5 $O/parity_$v.txt; exit 1; }
  cat $O/parity_$v.txt
done
for r in 1 2; do for v in fast mixed; do
  timeout -k 10 200 python3 -u bench.py --variant $v --no-cpu-baseline --no-main05 > $O/bench_$v.$r.json 2> $O/bench_$v.$r.err || { tail -5 $O/bench_$v.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$v.$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', d['value'], 'ev', r['kernel_avg_us'], 'roll', d['rollout']['us_per_step'], 'ppo', d['ppo_rollout']['us_per_step'])"
done; done
AB_DIR=tools/ab bash tools/ab_ppo_prof.sh 2>&1 | grep -E "a_base|e_vpf0" | tee $O/ab_ppo.txt
timeout -k 10 120 python3 tools/exp_stamps_split.py --lib tools/st/stamps.so > $O/stamps.txt 2>&1 || { tail -5 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/pmc -o sq64 --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2> $O/pmc_sq64.err || { echo "sq64 pmc rc=$?"; tail -5 $O/pmc_sq64.err; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d $O/pmc -o sqmix --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline --no-rollout > /dev/null 2> $O/pmc_sqmix.err || { echo "sqmix pmc rc=$?"; tail -5 $O/pmc_sqmix.err; }
find $O/pmc -name "*counter_collection.csv" | head
