#!/bin/bash
# round 6 (s): the plane-GEMM alternates' float64 test, then the full GPU suite and smoke()
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_h3.py \
    -k planes_vs_float64 > gpurun_out/r06s_planes.log 2>&1; rc=$?
tail -3 gpurun_out/r06s_planes.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r06s_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r06s_pytest_gpu.log; grep -E "FAIL|Error" gpurun_out/r06s_pytest_gpu.log | head -10
exit $rc
