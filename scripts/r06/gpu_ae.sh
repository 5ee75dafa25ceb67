#!/bin/bash
# round 6 (ae): rows in flight per thread in the heads' backward (k_head_bwd: 4, round 5; 8): its tests with 8, then
# one update replayed per setting (one process each)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
MERLIN_HEAD_ROWS=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_head.py \
    tests/test_gpu_dz_planes.py tests/test_gpu_fast_step.py > gpurun_out/r06ae_tests.log 2>&1; rc=$?
echo "tests rows 8: $(tail -1 gpurun_out/r06ae_tests.log)"; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
for N in 4 8 4 8; do
  MERLIN_HEAD_ROWS=$N timeout -k 10 300 python -u scripts/ab_update.py 3 4 fast_timers4 > gpurun_out/r06ae_ab$N.log 2>&1; rc=$?
  echo "rows $N: $(grep -o 'median [0-9.]* ms/update' gpurun_out/r06ae_ab$N.log)"; grep -E "k_head_bwd" gpurun_out/r06ae_ab$N.log | head -2
  crash $rc && exit $rc
done
exit 0
