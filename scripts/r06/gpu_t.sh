#!/bin/bash
# round 6 (t): the final tree -- the driver-settings bench under rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE
# passes of the same command, step sequence, busy union), then the driver-settings bench line with every tier
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
TAG=r06t PMC=1 bash scripts/gpu_profile_bench.sh > gpurun_out/r06t_prof.log 2>&1; rc=$?
tail -5 gpurun_out/r06t_prof.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06t_bench_driver.log 2>&1; rc=$?
tail -c 1500 gpurun_out/r06t_bench_driver.log; exit $rc
