#!/bin/bash
# Iteration check on the GPU box: selected GPU tests (TESTS, default all gpu tests), then a
# short bench (BENCH_ARGS).  Each step bounded; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_iter.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 2 --no-cpu-baseline --no-tiers} > gpurun_out/bench_iter.log 2>&1
rc=$?; tail -3 gpurun_out/bench_iter.log; exit $rc
