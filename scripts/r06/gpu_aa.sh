#!/bin/bash
# round 6 (aa): FOMAML's conv3 phase on 128-bit LDS reads (the same bits): its tests and the tier, then a trace of it
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fomaml.py \
    tests/test_gpu_grouped_policy.py > gpurun_out/r06aa_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06aa_tests.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 10 --warmup 3 > gpurun_out/r06aa_fomaml.log 2>&1; rc=$?
tail -1 gpurun_out/r06aa_fomaml.log; crash $rc && exit $rc
BENCH_ARGS="--fomaml --steps 10 --warmup 3" TAG=r06aa_fomaml PMC_TIMED_FRAC=1 bash scripts/gpu_profile_bench.sh > gpurun_out/r06aa_prof.log 2>&1; rc=$?
head -14 gpurun_out/summary/r06aa_fomaml_kernel_stats.md; exit $rc
