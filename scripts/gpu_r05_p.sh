#!/bin/bash
# round 5 (p): planes / loss tests, per-step timelines, one-setting-per-process A/B
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dz_planes.py \
    tests/test_gpu_loss.py tests/test_gpu_fast_step.py > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05p_tests.log; [ $rc -ne 0 ] && exit $rc
AB="${AB:-fast fast_nodzp}" bash scripts/gpu_r05_n.sh > gpurun_out/r05p_timelines.log 2>&1 || exit $?
grep -A4 "^==" gpurun_out/r05p_timelines.log
AB="${AB2:-fast fast_nodzp fast fast_nodzp}" bash scripts/gpu_r05_m.sh
