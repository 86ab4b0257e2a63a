#!/bin/bash
# round 4: the sub-step / PPO parity tests, then one bench line (each GPU step under its own timeout)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r04a}; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_split.py tests/test_gpu_ppo.py tests/test_gpu_episode_replay.py} > $O/pytest.log 2>&1
rc=$?; tail -25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -5 $O/bench.err; exit $rc
