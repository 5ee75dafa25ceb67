#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_update_grad.py \
    tests/test_gpu_fomaml.py > gpurun_out/r06h_grad.log 2>&1; rc=$?
grep -E "vs float64|ties|PASS|FAIL|Error|passed|failed" gpurun_out/r06h_grad.log | tail -50; exit $rc
