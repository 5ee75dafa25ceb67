#!/bin/bash
# round 6 (z): head-gradient, logit and head-weight loads issued unconditionally (k_head_bwd, k_ppo_loss, k_group_fc1):
# their tests, then the driver-settings bench (no tiers) and the FOMAML tier
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_head.py \
    tests/test_gpu_loss.py tests/test_gpu_fast_step.py tests/test_gpu_update_benched.py tests/test_gpu_update_grad.py \
    tests/test_gpu_dz_planes.py tests/test_gpu_fomaml.py tests/test_gpu_grouped_policy.py tests/test_gpu_ppo.py tests/test_gpu_stage_precision.py \
    > gpurun_out/r06z_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06z_tests.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-tiers --no-cpu-baseline > gpurun_out/r06z_bench.log 2>&1; rc=$?
grep -o '"value": [0-9.]*\|"phases_ms": {[^}]*}' gpurun_out/r06z_bench.log | head -2
grep -o '"k_head_bwd": {"launches[^}]*}\|"k_ppo_loss": {"launches[^}]*}\|"gemm_fc1_dgrad": {"launches[^}]*}' gpurun_out/r06z_bench.log
crash $rc && exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 10 --warmup 3 > gpurun_out/r06z_fomaml.log 2>&1; rc=$?
tail -1 gpurun_out/r06z_fomaml.log; exit $rc
