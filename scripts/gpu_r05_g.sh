#!/bin/bash
# round 5 (g): operand-planes tests, then the in-process A/B of the update switches
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dz_planes.py \
    tests/test_gpu_loss.py tests/test_gpu_fast_step.py tests/test_gpu_windows.py > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r05g_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/ab_update.py 3 5 ${AB:-fast,fast_noa3p,fast_nodzp,fast_h3t1} > gpurun_out/r05g_ab.log 2>&1
rc=$?; tail -12 gpurun_out/r05g_ab.log; exit $rc
