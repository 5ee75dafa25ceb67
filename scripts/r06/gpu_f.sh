#!/bin/bash
# round 6 (f): reference-gradient tests (stored reference advantages), FOMAML tests + tier with side-stream refills,
# h3 GEMM tests after the probe gating
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_update_grad.py \
    > gpurun_out/r06f_grad.log 2>&1; rc=$?
grep -E "reference|PASS|FAIL|Error|passed|failed" gpurun_out/r06f_grad.log | tail -28; crash $rc && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fomaml.py \
    tests/test_gpu_grouped_policy.py tests/test_gpu_h3.py tests/test_gpu_cli.py > gpurun_out/r06f_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r06f_tests.log; crash $rc && exit $rc
timeout -k 10 300 python -u scripts/probe_fomaml.py 4 > gpurun_out/r06f_fomaml_phases.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/r06f_fomaml_phases.log; crash $rc && exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 5 --warmup 2 > gpurun_out/r06f_fomaml_bench.log 2>&1; rc=$?
tail -c 600 gpurun_out/r06f_fomaml_bench.log
