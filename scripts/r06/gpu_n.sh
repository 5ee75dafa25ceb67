#!/bin/bash
# round 6 (n): which multi-stream capture shapes survive hipStreamEndCapture -- lanes without nested refill streams
# (pure torch, then PPO's lanes with in-lane refills), then the rollout A/B with in-lane refills
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for m in a1; do
  timeout -k 10 120 python -u scripts/probe_lane_capture.py $m 2 > gpurun_out/r06n_$m.log 2>&1; rc=$?
  echo "== $m rc=$rc"; grep -v '^  File "/usr' gpurun_out/r06n_$m.log | tail -4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
