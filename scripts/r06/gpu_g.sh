#!/bin/bash
# round 6 (g): the whole -m gpu suite, then the driver-settings bench under rocprofv3 (kernel trace + FETCH_SIZE /
# WRITE_SIZE passes of the same command)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r06g_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r06g_pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/r06g_pytest_gpu.log | head -5
[ $rc -ne 0 ] && exit $rc
TAG=r06g PMC=1 bash scripts/gpu_profile_bench.sh
