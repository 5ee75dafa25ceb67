#!/bin/bash
# round 6 (ad): the per-step look-ahead refill over 4 envs per lane (16 one-wave blocks at 4,096 envs) against 16 (4
# blocks): the env / rollout tests with span 4, then the rollout at the bench state per span (one process each)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
MERLIN_REFILL_SPAN=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_env.py \
    tests/test_gpu_rollout_graph.py > gpurun_out/r06ad_tests.log 2>&1; rc=$?
echo "tests span 4: $(tail -1 gpurun_out/r06ad_tests.log)"; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
for S in 16 4 16 4; do
  MERLIN_REFILL_SPAN=$S WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06ad_span$S.log 2>&1; rc=$?
  echo "span $S: $(tail -1 gpurun_out/r06ad_span$S.log)"; crash $rc && exit $rc
done
exit 0
