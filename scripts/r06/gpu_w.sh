#!/bin/bash
# round 6 (w): the fused draw + env step with every head-partial and bias load issued up front (its own
# instantiation; the plain step down to 105 VGPRs): env / rollout / FOMAML / DP tests, then the FOMAML tier, the
# rollout at the bench state and the env-only tiers
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_env.py \
    tests/test_gpu_rollout_graph.py tests/test_gpu_fomaml.py tests/test_gpu_grouped_policy.py tests/test_gpu_hard22.py \
    tests/test_gpu_act.py tests/test_gpu_eval.py tests/test_gpu_dp.py > gpurun_out/r06w_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06w_tests.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 10 --warmup 3 > gpurun_out/r06w_fomaml.log 2>&1; rc=$?
tail -1 gpurun_out/r06w_fomaml.log; crash $rc && exit $rc
WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06w_rollout.log 2>&1; rc=$?
tail -1 gpurun_out/r06w_rollout.log; crash $rc && exit $rc
timeout -k 10 300 python -u bench.py --env-tier-only > gpurun_out/r06w_env.log 2>&1; rc=$?
tail -c 600 gpurun_out/r06w_env.log; exit $rc
