#!/bin/bash
# round 6 (x): frames per block of the acting conv3 (k_codes_conv3<CC_F>: 4 = 4.5 gather rounds per thread, 2, 1),
# one process each at the bench state, then its parity tests with the winner
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for F in 4 8 16 4; do
  MERLIN_CC_F=$F WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06x_ccf$F.log 2>&1; rc=$?
  echo "CC_F=$F: $(tail -1 gpurun_out/r06x_ccf$F.log)"; crash $rc && exit $rc
done
for F in 8 16; do
  MERLIN_CC_F=$F timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_rollout_graph.py > gpurun_out/r06x_tests$F.log 2>&1; rc=$?
  echo "tests CC_F=$F: $(tail -1 gpurun_out/r06x_tests$F.log)"; crash $rc && exit $rc
done
exit 0
