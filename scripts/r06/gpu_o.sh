#!/bin/bash
# round 6 (o): the rollout A/B -- one chain with side-stream refills (l1) against 2 / 4 env-range lanes with in-lane
# refills -- at the bench workload
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
WARM=6 timeout -k 10 400 python -u scripts/probe_rollout.py 5 l1,l2,l4 > gpurun_out/r06o_rollout.log 2>&1; rc=$?
tail -5 gpurun_out/r06o_rollout.log; exit $rc
