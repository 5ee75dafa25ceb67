#!/bin/bash
# round 6 (ab): outputs per thread and gather round in the acting conv3 (k_codes_conv3<CC_U>; 1 = one output's 9
# gathers at a time, the round-5 form), one process each at the bench state, then the rollout tests
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for U in 1 2 3 5 1 2; do
  MERLIN_CC_U=$U WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06ab_ccu$U.log 2>&1; rc=$?
  echo "CC_U=$U: $(tail -1 gpurun_out/r06ab_ccu$U.log)"; crash $rc && exit $rc
done
for U in 2 3 5; do
  MERLIN_CC_U=$U timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_rollout_graph.py > gpurun_out/r06ab_tests$U.log 2>&1; rc=$?
  echo "tests CC_U=$U: $(tail -1 gpurun_out/r06ab_tests$U.log)"; crash $rc && exit $rc
done
exit 0
