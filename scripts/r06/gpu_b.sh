#!/bin/bash
# round 6 (b): the new parity tests (reference gradient, bad-tile flag, cfg 3's workload as 8 ranks x 4096 envs,
# FOMAML's grouped acting step), then the driver-settings bench with the weight gradient on the main stream
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_update_grad.py \
    tests/test_gpu_rollout_graph.py tests/test_gpu_grouped_policy.py tests/test_gpu_fomaml.py \
    > gpurun_out/r06b_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|worst|differ|passed|failed" gpurun_out/r06b_tests.log | tail -40; crash $rc && exit $rc
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread tests/test_gpu_dp.py \
    tests/test_gpu_bench_dp.py > gpurun_out/r06b_dp.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|cfg 3|passed|failed" gpurun_out/r06b_dp.log | tail -25; crash $rc && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r06b_bench.log 2>&1 || { tail -30 gpurun_out/r06b_bench.log; exit 1; }
tail -c 3000 gpurun_out/r06b_bench.log
