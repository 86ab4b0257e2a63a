#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/prof
R=$PWD; TAG=${TAG:-r01b}
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in fast faithful; do
  timeout -k 10 200 python bench.py --variant $v --no-cpu-baseline > gpurun_out/bench_${TAG}_$v.json 2>>gpurun_out/bench_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/$TAG -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_trace_$TAG.json 2>>$R/gpurun_out/prof_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $R/gpurun_out/prof/$TAG -o pmc_sq --output-format csv -- python3 $R/bench.py --eager --steps 30 --warmup 5 --no-cpu-baseline > /dev/null 2>>$R/gpurun_out/prof_$TAG.err || echo "sq pmc failed rc=$?"
ls $R/gpurun_out/prof/$TAG
