#!/bin/bash
# round 6 (d): the reference-gradient tests (injected reference advantages / own normalisation), the env and rollout
# tests after the fallback change, the rollout A/B with and without the fallback pass, the driver-settings bench
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_update_grad.py \
    > gpurun_out/r06d_grad.log 2>&1; rc=$?
grep -E "weight|bias|PASS|FAIL|Error|passed|failed" gpurun_out/r06d_grad.log | tail -45; crash $rc && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_env.py \
    tests/test_gpu_rollout_graph.py tests/test_gpu_hard22.py tests/test_gpu_ppo.py tests/test_gpu_act_step.py \
    > gpurun_out/r06d_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06d_tests.log; crash $rc && exit $rc
timeout -k 10 300 python -u scripts/probe_rollout.py 5 1,1fb > gpurun_out/r06d_rollout.log 2>&1 \
    || { tail -20 gpurun_out/r06d_rollout.log; exit 1; }
tail -3 gpurun_out/r06d_rollout.log
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06d_bench.log 2>&1 \
    || { tail -30 gpurun_out/r06d_bench.log; exit 1; }
tail -c 1500 gpurun_out/r06d_bench.log
