#!/bin/bash
# round 5 (j): operand-planes tests, then a kernel trace of the update A/B setting(s)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dz_planes.py \
    tests/test_gpu_loss.py > gpurun_out/r05j_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r05j_tests.log; [ $rc -ne 0 ] && exit $rc
AB=${AB:-fast} LOG=${LOG:-r05j} bash scripts/gpu_r05_i.sh
