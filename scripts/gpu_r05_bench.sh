#!/bin/bash
# round 5: the driver's bench command (defaults: every tier + the CPU baseline), log under gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py ${BENCH_ARGS} > gpurun_out/${LOG:-r05_bench_driver}.log 2>&1
rc=$?; tail -c 600 gpurun_out/${LOG:-r05_bench_driver}.log; exit $rc
