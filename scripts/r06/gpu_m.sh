#!/bin/bash
# round 6 (m): the rollout as env-range lanes on concurrent streams: the rollout / env / DP tests, then the rollout
# A/B (1 / 2 / 4 lanes) at the bench workload
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rollout_graph.py \
    tests/test_gpu_env.py tests/test_gpu_capture_safety.py tests/test_gpu_hard22.py > gpurun_out/r06m_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06m_tests.log; grep -E "FAIL|Error" gpurun_out/r06m_tests.log | head; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
WARM=6 timeout -k 10 400 python -u scripts/probe_rollout.py 5 l1,l2,l4 > gpurun_out/r06m_rollout.log 2>&1; rc=$?
tail -5 gpurun_out/r06m_rollout.log; exit $rc
