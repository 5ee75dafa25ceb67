#!/bin/bash
# round 6 (k): the one-accumulator GEMM probes; FOMAML with no refill / fallback nodes in reseed mode (its tests, then
# the FOMAML bench tier)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 200 python -u scripts/probe_one_acc.py 111000 20 > gpurun_out/r06k_one_acc.log 2>&1; rc=$?
cat gpurun_out/r06k_one_acc.log; crash $rc && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fomaml.py \
    tests/test_gpu_grouped_policy.py tests/test_gpu_env.py > gpurun_out/r06k_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06k_tests.log; crash $rc && exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 10 --warmup 3 > gpurun_out/r06k_fomaml.log 2>&1; rc=$?
tail -3 gpurun_out/r06k_fomaml.log; exit $rc
