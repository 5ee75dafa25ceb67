#!/bin/bash
# round 6 (v): the batched trainer on flattened observations (observation.flatten / fully_observable -> MLP), and the
# env / eval / CLI / PPO tests around it
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_flat_obs.py \
    tests/test_gpu_env.py tests/test_gpu_eval.py tests/test_gpu_cli.py tests/test_gpu_ppo.py > gpurun_out/r06v_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r06v_tests.log; grep -E "FAIL|Error" gpurun_out/r06v_tests.log | head -20; exit $rc
