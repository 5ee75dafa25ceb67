#!/bin/bash
# round 6 (i): the compact R pass -- its tests, the fast step's parity tests, then an in-process A/B
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_patch_compact.py tests/test_gpu_fast_step.py tests/test_gpu_windows.py \
    tests/test_gpu_update_benched.py tests/test_gpu_dz_planes.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r06i_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r06i_tests.log; grep -E "FAILED|Error|assert" gpurun_out/r06i_tests.log | head -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_update.py 4 6 fast,fast_nocompact,fast_cgather,fast_timers4,fast_nocompact_timers4 \
    > gpurun_out/r06i_ab.log 2>&1; rc=$?
cat gpurun_out/r06i_ab.log | grep -v "^W2026\|^E2026" | head -60
exit $rc
