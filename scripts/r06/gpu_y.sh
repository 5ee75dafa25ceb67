#!/bin/bash
# round 6 (y): the heads epilogues' weight loads issued unconditionally: the GEMM / rollout tests, the rollout at the
# bench state, then the driver-settings bench line (no tiers)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_h3.py \
    tests/test_gpu_dz_planes.py tests/test_gpu_rollout_graph.py tests/test_gpu_fast_step.py \
    tests/test_gpu_update_benched.py > gpurun_out/r06y_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06y_tests.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06y_rollout.log 2>&1; rc=$?
tail -1 gpurun_out/r06y_rollout.log; crash $rc && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-tiers --no-cpu-baseline > gpurun_out/r06y_bench.log 2>&1; rc=$?
grep -o '"value": [0-9.]*\|"phases_ms": {[^}]*}' gpurun_out/r06y_bench.log | head -3; exit $rc
