#!/bin/bash
# round 6 (ac): representatives per 16-lane group and gather round in the update's conv3 (k_window_conv3_reps<NR>,
# 1 = round 5's one row at a time): the windows tests for each, then one update replayed per setting (one process each)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for N in 2 3; do
  MERLIN_REPS_NR=$N timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_windows.py \
      tests/test_gpu_fast_step.py tests/test_gpu_dz_planes.py > gpurun_out/r06ac_tests$N.log 2>&1; rc=$?
  echo "tests NR=$N: $(tail -1 gpurun_out/r06ac_tests$N.log)"; crash $rc && exit $rc
  [ $rc -ne 0 ] && exit $rc
done
for N in 1 2 3 1 2 3; do
  MERLIN_REPS_NR=$N timeout -k 10 300 python -u scripts/ab_update.py 3 4 fast_timers4 > gpurun_out/r06ac_ab$N.log 2>&1; rc=$?
  echo "NR=$N: $(head -3 gpurun_out/r06ac_ab$N.log | tr '\n' ' ')"; grep -E "conv3|k_window" gpurun_out/r06ac_ab$N.log | head -3
  crash $rc && exit $rc
done
exit 0
